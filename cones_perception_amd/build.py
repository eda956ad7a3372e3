"""Build the gfx950 C-ABI library (libcones_gpu.so) in-tree with hipcc.

The .so lands in cones_perception_amd/lib/ (git-ignored, shipped to the GPU box with the
snapshot). Device and host code are compiled with -ffp-contract=off: the reference is a
non-FMA x86-64 build and the kernels must round exactly like it.
"""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(PKG, "build")
LIB = os.path.join(PKG, "lib", "libcones_gpu.so")
ROOT = os.path.dirname(PKG)
ARCH = os.environ.get("CG_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", f"--offload-arch={ARCH}",
             "-Wall", "-Wno-unused-function", "-I", os.path.join(ROOT, "include")]
HEADERS = [os.path.join(CSRC, h) for h in ("cg_math.h", "cg_sort.h", "cg_internal.h", "cg_device.h", "cg_pcl.h",
                                            "cg_backend.h", "cg_grid.h", "cg_host.h")] + \
          [os.path.join(ROOT, "include", "cones_gpu.h")]


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"build step failed: {' '.join(cmd[:3])} ...")
    return r


def build(verbose=False, force=False):
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    objs = []
    src = os.path.join(CSRC, "cg_synth.c")
    o = os.path.join(OBJ, "cg_synth.o")
    if force or _stale(o, [src] + HEADERS):
        _run(["gcc", "-O2", "-fPIC", "-ffp-contract=off", "-std=c11", "-Wall", "-c", src, "-o", o], verbose)
    objs.append(o)
    jobs = []
    for name in ("cg_kernels.hip", "cg_large.hip", "cg_recrop.hip", "cg_colornet.hip", "cg_api.cpp", "cg_host.cpp",
                 "cg_track.cpp"):
        src = os.path.join(CSRC, name)
        o = os.path.join(OBJ, name.rsplit(".", 1)[0] + ".o")
        if force or _stale(o, [src] + HEADERS):
            jobs.append([HIPCC, "-x", "hip", *HIP_FLAGS, "-c", src, "-o", o])
        objs.append(o)
    if jobs:   # the translation units compile independently (hipcc is single-threaded)
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(min(len(jobs), max(1, (os.cpu_count() or 1)))) as ex:
            list(ex.map(lambda c: _run(c, verbose), jobs))
    if force or _stale(LIB, objs):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB, *objs, "-lpthread"], verbose)
    return LIB


def build_host_demo(verbose=False):
    """g++ build of the C++ node mirror demo (host/nodes_demo.cpp) against libcones_gpu.so."""
    lib = build(verbose)
    out = os.path.join(PKG, "lib", "nodes_demo")
    src = os.path.join(PKG, "host", "nodes_demo.cpp")
    if _stale(out, [src, os.path.join(PKG, "host", "cones_nodes.hpp"), lib]):
        _run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-I", os.path.join(PKG, "host"),
              src, "-o", out, "-L", os.path.dirname(lib), "-lcones_gpu",
              "-Wl,-rpath,$ORIGIN"], verbose)
    return out


def build_probes(verbose=False):
    """hipcc builds of the sort probes (tools/pcl_probe.hip, tools/pcl_leaf_probe.hip): the
    device PCL sort against libstdc++'s std::sort, run by tests/test_gpu_pcl_probe.py."""
    csrc = os.path.join(PKG, "csrc")
    deps = [os.path.join(csrc, h) for h in os.listdir(csrc) if h.endswith(".h")]
    outs = []
    for name in ("pcl_probe", "pcl_leaf_probe"):
        src = os.path.join(ROOT, "tools", name + ".hip")
        out = os.path.join(PKG, "lib", name)
        if _stale(out, [src] + deps):
            _run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950",
                  "-w", "-I", os.path.join(ROOT, "include"), src, "-o", out], verbose)
        outs.append(out)
    return outs


def build_oracle(verbose=False):
    """Compile the CPU restatement (test infrastructure, oracle/)."""
    _run(["make", "-C", os.path.join(ROOT, "oracle")], verbose)
    return os.path.join(ROOT, "oracle", "build", "libcg_oracle.so")


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
    print(build_oracle(verbose=True))
    print(build_host_demo(verbose=True))
    print(build_probes(verbose=True))
