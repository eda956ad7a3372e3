"""The device PCL voxel sort (csrc/cg_pcl.h) against libstdc++'s own std::sort on the GPU, with
no oracle in between: tools/pcl_probe.hip (the frame kernel's LDS form: 4,000 random, tie-heavy,
sorted, reversed and organ-pipe cases of up to 2,048 records; every seventh case starts with a
depth budget of 0-3, checked against libstdc++'s __introsort_loop + __final_insertion_sort with
that budget, so the heapsort fallbacks run) and tools/pcl_leaf_probe.hip (the large path's leaf
configuration: up to 4,096 records, 8 per thread; every seventh case with a spent budget too).
Built by build() into the package's lib/."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "cones_perception_amd", "lib")


@pytest.mark.gpu
@pytest.mark.parametrize("exe,args", [
    ("pcl_probe", ["4000", "243"]),
    ("pcl_probe", ["300", "1500"]),
    ("pcl_leaf_probe", ["400", "4096", "9"]),
    ("pcl_leaf_probe", ["100", "4096", "1000"]),
])
def test_device_sort_matches_libstdcxx(exe, args):
    path = os.path.join(LIB, exe)
    assert os.path.exists(path), f"{path} missing: run __graft_entry__.build()"
    r = subprocess.run([path] + args, capture_output=True, text=True, timeout=90)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 mismatches" in r.stdout, r.stdout
