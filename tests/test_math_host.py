"""Host compile of the device restatements (csrc/cg_math.h, csrc/cg_sort.h) checked against
the host glibc and libstdc++ they restate: atan2f/atanf bit for bit, the exact-threshold
helpers, and std::sort's permutation on tie-heavy inputs."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "cones_perception_amd", "csrc")

PROG = r'''
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <algorithm>
#include <random>
#include <vector>
#include "cg_math.h"
#include "cg_sort.h"
int main() {
  std::mt19937_64 rng(12345);
  long bad = 0;
  // atan2f: random bit patterns, scaled normals, axis and sector-boundary neighbourhoods
  for (long i = 0; i < 4000000; i++) {
    float y, x;
    uint64_t r = rng();
    switch (i & 3) {
      case 0: y = cg_bitsf((uint32_t)r); x = cg_bitsf((uint32_t)(r >> 32)); break;
      case 1: y = (float)((int32_t)r) * 1e-8f; x = (float)((int32_t)(r >> 32)) * 1e-8f; break;
      case 2: { double a = (double)(r % 17) * 22.0 * M_PI / 180.0 + ((double)(r >> 40) / 1.7e13 - 0.5) * 1e-5;
                x = (float)(5.0 * cos(a)); y = (float)(5.0 * sin(a)); break; }
      default: y = (r & 1) ? 0.0f : -0.0f; x = cg_bitsf((uint32_t)(r >> 32)); break;
    }
    float a = atan2f(y, x), b = cg_atan2f(y, x);
    if (!(std::isnan(a) && std::isnan(b)) && cg_fbits(a) != cg_fbits(b)) bad++;
  }
  if (bad) { printf("atan2f mismatches %ld\n", bad); return 1; }
  // exact compare helpers: (double)z < t  <=>  z < ceil_to_float(t); (double)z <= t <=> z <= floor_to_float(t)
  for (long i = 0; i < 2000000; i++) {
    double t = ((double)(int64_t)rng() / 9.2e18) * 20.0;
    float c = cg_ceil_to_float(t), f = cg_floor_to_float(t);
    float zs[3] = {c, cg_next_down(c), (float)t};
    for (float z : zs) {
      if (((double)z < t) != (z < c)) bad++;
      if (((double)z <= t) != (z <= f)) bad++;
    }
  }
  if (bad) { printf("threshold helper mismatches %ld\n", bad); return 2; }
  // sector of the exact angle vs the reference expression
  for (long i = 0; i < 2000000; i++) {
    float y = (float)((int32_t)rng()) * 1e-9f, x = (float)((int32_t)rng()) * 1e-9f;
    float at = atan2f(y, x);
    float ang = (at < 0) ? at += 2 * M_PI : at;
    int ref = std::isnan(ang) ? 17 : (int)floorf(ang / (float)(22 * M_PI / 180));
    if (ref != cg_sector(cg_atan2f(y, x))) bad++;
  }
  if (bad) { printf("sector mismatches %ld\n", bad); return 3; }
  // std::sort permutation restatement
  struct R { unsigned key, id; };
  for (int it = 0; it < 20000; it++) {
    int n = (it % 5 == 0) ? (int)(rng() % 3000) : (int)(rng() % 120);
    unsigned kr = 1 + (unsigned)(rng() % ((it % 2) ? 4 : 1000));
    std::vector<R> a(n);
    for (int i = 0; i < n; i++) a[i] = {(unsigned)(rng() % kr), (unsigned)i};
    auto b = a;
    auto lt = [](const R& p, const R& q) { return p.key < q.key; };
    std::sort(a.begin(), a.end(), lt);
    int stk[3 * CG_SORT_STACK];
    cg_std_sort(b.data(), (long)n, lt, stk);
    for (int i = 0; i < n; i++) if (a[i].id != b[i].id) { bad++; break; }
  }
  if (bad) { printf("sort mismatches %ld\n", bad); return 4; }
  printf("ok\n");
  return 0;
}
'''


def test_device_restatements_on_host(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text(PROG)
    exe = tmp_path / "t"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", CSRC, str(src), "-o", str(exe)],
                   check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr
