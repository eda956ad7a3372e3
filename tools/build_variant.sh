#!/bin/bash
# Build an experimental variant of libcones_gpu.so with extra defines for the kernel
# translation unit (e.g. -DCG_BLOCK=1024) into lib_variants/<name>/; select it at run time
# with CONES_GPU_LIB=lib_variants/<name>/libcones_gpu.so. The default build is untouched.
# API_FLAGS adds defines for cg_api.cpp as well (e.g. API_FLAGS=-DCG_SPIN_SYNC).
set -e
name=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/lib_variants/$name
mkdir -p "$O"
F="-x hip -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -Wall -Wno-unused-function -I $R/include"
C=$R/cones_perception_amd/csrc
/opt/rocm/bin/hipcc $F "$@" -c $C/cg_kernels.hip -o $O/cg_kernels.o &
/opt/rocm/bin/hipcc $F "$@" -c ${LARGE_SRC:-$C/cg_large.hip} -o $O/cg_large.o &
/opt/rocm/bin/hipcc $F -c $C/cg_recrop.hip -o $O/cg_recrop.o &
/opt/rocm/bin/hipcc $F -c $C/cg_colornet.hip -o $O/cg_colornet.o &
/opt/rocm/bin/hipcc $F -c $C/cg_track.cpp -o $O/cg_track.o &
/opt/rocm/bin/hipcc $F ${API_FLAGS:-} -c $C/cg_api.cpp -o $O/cg_api.o &
/opt/rocm/bin/hipcc $F -c $C/cg_host.cpp -o $O/cg_host.o &
gcc -O2 -fPIC -ffp-contract=off -std=c11 -Wall -c $C/cg_synth.c -o $O/cg_synth.o
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $O/libcones_gpu.so $O/*.o -lpthread
rm -f $O/*.o
echo "$O/libcones_gpu.so"
