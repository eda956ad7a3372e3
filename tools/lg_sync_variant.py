"""Debug variant of the large path: every launch in cg_large.hip is followed by a stream
synchronisation that reports the first failing launch (source line) on stderr. Builds
lib_variants/lgsync/libcones_gpu.so (select with CONES_GPU_LIB)."""
import os
import re
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(R, "cones_perception_amd/csrc/cg_large.hip")).read()
out, i = [], 0
for m in re.finditer(r"hipLaunchKernelGGL\(", src):
    if m.start() < i:
        continue
    j, depth = m.end(), 1
    while depth:
        depth += {"(": 1, ")": -1}.get(src[j], 0)
        j += 1
    assert src[j] == ";"
    line = src.count("\n", 0, m.start()) + 1
    out.append(src[i:j + 1])
    out.append(f' {{ hipError_t e_ = hipStreamSynchronize(s); if (e_ != hipSuccess) '
               f'fprintf(stderr, "LGDBG launch at cg_large.hip:{line}: %s\\n", hipGetErrorString(e_)); }}')
    i = j + 1
out.append(src[i:])
dst = os.path.join(R, "lib_variants", "lgsync_src")
os.makedirs(dst, exist_ok=True)
open(os.path.join(dst, "cg_large.hip"), "w").write("#include <cstdio>\n" + "".join(out))
env = dict(os.environ, LARGE_SRC=os.path.join(dst, "cg_large.hip"))
print(subprocess.run(["bash", os.path.join(R, "tools", "build_variant.sh"), "lgsync",
                      f"-I{os.path.join(R, 'cones_perception_amd/csrc')}"], capture_output=True, text=True, env=env).stdout)
