"""The workgroup PCL voxel sort (cg_pcl.h pcl_block_sort) modelled thread by thread on the host
(tests/pb_model.py, every array access bounds-checked) against libstdc++'s std::sort: the
model's reference (pb_model.std_sort, a restatement of cg_sort.h) is itself pinned to the host
g++ std::sort on the same inputs."""
import os
import random
import subprocess

import pytest

import pb_model as M

PROG = r'''
#include <algorithm>
#include <cstdio>
#include <vector>
int main() {
  int cases;
  if (scanf("%d", &cases) != 1) return 1;
  for (int c = 0; c < cases; c++) {
    int n; scanf("%d", &n);
    std::vector<unsigned long long> a(n);
    for (auto& x : a) scanf("%llu", &x);
    std::sort(a.begin(), a.end(), [](unsigned long long p, unsigned long long q) { return (p >> 32) < (q >> 32); });
    for (auto x : a) printf("%llu ", x);
    printf("\n");
  }
  return 0;
}
'''


def _cases(seed, count, nmax):
    rng = random.Random(seed)
    out = []
    for it in range(count):
        n = rng.choice([0, 1, 16, 17, 64, 65, 128, 243, 256, 511, nmax]) if it % 2 else rng.randrange(0, nmax + 1)
        kr = rng.choice([1, 2, 3, 4, 10, 60, 1000, 100000])
        k = [rng.randrange(kr) for _ in range(n)]
        if it % 11 == 1:
            k.sort()
        if it % 13 == 2:
            k.sort(reverse=True)
        if it % 17 == 3:
            k = [min(i, n - i) for i in range(n)]
        out.append([(k[i] << 32) | i for i in range(n)])
    return out


def test_std_sort_restatement_matches_gxx(tmp_path):
    src = tmp_path / "s.cpp"
    src.write_text(PROG)
    exe = tmp_path / "s"
    subprocess.run(["g++", "-O2", "-std=c++17", str(src), "-o", str(exe)], check=True)
    cases = _cases(11, 150, 2048)
    inp = f"{len(cases)}\n" + "".join(f"{len(a)} " + " ".join(map(str, a)) + "\n" for a in cases)
    r = subprocess.run([str(exe)], input=inp, capture_output=True, text=True, check=True)
    lines = r.stdout.split("\n")
    for a, line in zip(cases, lines):
        assert [int(x) for x in line.split()] == M.std_sort(a)


@pytest.mark.parametrize("seed,nmax", [(1, 512), (2, 1024), (3, 2048), (6, 4096)])
def test_block_sort_model_matches_std_sort(seed, nmax):
    for i, a in enumerate(_cases(seed, 40, nmax)):
        assert M.block_sort(a, oop=bool(i & 1)) == M.std_sort(a), len(a)


def test_block_sort_model_heapsort_fallback():
    # small depth budgets force the __partial_sort branch at several levels
    rng = random.Random(3)
    for it in range(40):
        n = rng.randrange(17, 1100)
        kr = rng.choice([2, 5, 100, 10000])
        a = [(rng.randrange(kr) << 32) | i for i in range(n)]
        d = it % 4
        assert M.block_sort(a, depth0=d) == M.std_sort(a, depth0=d), (n, d)


@pytest.mark.parametrize("seed", [4, 5])
def test_partition_levels_model_matches_std_sort(seed):
    """cg_large.hip's split/swap levels (small leaves so that several levels run) with the
    leaves through the block model, against std::sort's permutation."""
    rng = random.Random(seed)
    for it in range(6):
        n = rng.choice([300, 1000, 2500, 4000])
        kr = rng.choice([3, 40, 1000, 100000])
        k = [rng.randrange(kr) for _ in range(n)]
        if it == 2:
            k.sort()
        a = [(k[i] << 32) | i for i in range(n)]
        assert M.levels_sort(a, leaf=64) == M.std_sort(a), (n, kr)
        assert M.levels_sort(a, leaf=64, levels=3) == M.std_sort(a), (n, kr)   # long leaves


def test_wave_model_matches_std_sort():
    """cg_pcl.h pw_range64, lane by lane (tests/pb_model.wave_sort: all sub-ranges of a round
    partition together; L_k / R_k read from ds_permute lane tables; swaps as lane permutes; the
    swap count from one ballot counted over the sub-range) against std::sort on ranges of
    17-64, with every depth budget down to the heapsort fallback."""
    rng = random.Random(9)
    for it in range(1500):
        m = rng.randrange(17, 65)
        kr = rng.choice([1, 2, 3, 5, 20, 1000])
        a = [(rng.randrange(kr) << 32) | i for i in range(m)]
        if it % 7 == 0:
            a.sort()
        if it % 11 == 1:
            a.sort(reverse=True)
        d = 2 * M._lg(m) if it % 4 else rng.randrange(0, 4)
        assert M.wave_sort(a, d) == M.std_sort(a, depth0=d), (m, kr, d)


def test_chip_wide_leaf_stages_model():
    """cg_large.hip's leaf stages: a leaf's levels stop at 512-record ranges (lg_pcl_leaf), those
    stop at 64 (lg_pcl_mid), the rest one wave each (pw_range64); against std::sort."""
    rng = random.Random(12)
    for it in range(4):
        n = rng.choice([1500, 3000, 4096])
        kr = rng.choice([9, 300, 100000])
        a = [(rng.randrange(kr) << 32) | i for i in range(n)]
        assert M.levels_sort(a, leaf=4096) == M.std_sort(a), (n, kr)
        assert M.levels_sort(a, leaf=1024) == M.std_sort(a), (n, kr)
