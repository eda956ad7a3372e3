#!/bin/bash
# Build an experimental variant of libcones_gpu.so with extra defines for the kernel
# translation unit (e.g. -DCG_BLOCK=1024) into lib_variants/<name>/; select it at run time
# with CONES_GPU_LIB=lib_variants/<name>/libcones_gpu.so. The default build is untouched.
# API_FLAGS adds defines for cg_api.cpp as well. VARIANT=<header> force-includes an experiment
# header from tools/variants/ into every HIP translation unit (its CG_HOOK_* definitions replace
# the product's empty hooks, cg_internal.h), e.g.
#   VARIANT=tools/variants/exp_stop.h tools/build_variant.sh stop1 -DCG_EXP_STOP=1
set -e
name=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/lib_variants/$name
mkdir -p "$O"
INC=""
[ -n "${VARIANT:-}" ] && INC="-include $(cd "$(dirname "$VARIANT")" && pwd)/$(basename "$VARIANT")"
F="$INC -x hip -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -Wall -Wno-unused-function -I $R/include"
C=$R/cones_perception_amd/csrc
pids=()
/opt/rocm/bin/hipcc $F "$@" -c $C/cg_kernels.hip -o $O/cg_kernels.o & pids+=($!)
/opt/rocm/bin/hipcc $F "$@" -c ${LARGE_SRC:-$C/cg_large.hip} -o $O/cg_large.o & pids+=($!)
/opt/rocm/bin/hipcc $F -c $C/cg_recrop.hip -o $O/cg_recrop.o & pids+=($!)
/opt/rocm/bin/hipcc $F -c $C/cg_colornet.hip -o $O/cg_colornet.o & pids+=($!)
/opt/rocm/bin/hipcc $F -c $C/cg_track.cpp -o $O/cg_track.o & pids+=($!)
/opt/rocm/bin/hipcc $F ${API_FLAGS:-} -c $C/cg_api.cpp -o $O/cg_api.o & pids+=($!)
/opt/rocm/bin/hipcc $F -c $C/cg_host.cpp -o $O/cg_host.o & pids+=($!)
gcc -O2 -fPIC -ffp-contract=off -std=c11 -Wall -c $C/cg_synth.c -o $O/cg_synth.o
for p in "${pids[@]}"; do wait "$p"; done   # (set -e: a failed compile stops the build)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $O/libcones_gpu.so $O/*.o -lpthread
rm -f $O/*.o
echo "$O/libcones_gpu.so"
