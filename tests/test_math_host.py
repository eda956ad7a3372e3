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
#include <climits>
#include "cg_math.h"
#include "cg_sort.h"
struct R { unsigned key, id; };
// level-parallel model of std::sort's permutation (keys compared alone)
static void levels_sort(std::vector<R>& a) {
  const int n = (int)a.size();
  std::vector<char> head(n + 1, 0), heap(n, 0);
  head[0] = 1; head[n] = 1;
  struct Rg { int first, last, depth; };
  std::vector<Rg> act;
  if (n > 16) act.push_back({0, n, cg_lg(n) * 2});
  auto lt = [](const R& p, const R& q) { return p.key < q.key; };
  while (!act.empty()) {
    std::vector<Rg> nx;
    for (auto r : act) {
      if (r.depth == 0) {
        cg_heap_sort_range(a.data() + r.first, (long)(r.last - r.first), lt);
        for (int i = r.first; i < r.last; i++) heap[i] = 1;
        continue;
      }
      const int d = r.depth - 1, first = r.first, last = r.last, mid = first + (last - first) / 2;
      cg_move_median_to_first(a.data(), first, first + 1, mid, last - 1, lt);
      const unsigned p = a[first].key;
      std::vector<int> L, Rr;
      for (int i = first + 1; i < last; i++) if (a[i].key >= p) L.push_back(i);
      for (int i = last - 1; i > first; i--) if (a[i].key <= p) Rr.push_back(i);
      int s = 0;
      while (s < (int)L.size() && s < (int)Rr.size() && L[s] < Rr[s]) s++;
      const int cut = s == 0 ? L[0] : std::min(s < (int)L.size() ? L[s] : INT_MAX, Rr[s - 1]);
      for (int k = 0; k < s; k++) std::swap(a[L[k]], a[Rr[k]]);
      head[cut] = 1;
      if (cut - first > 16) nx.push_back({first, cut, d});
      if (last - cut > 16) nx.push_back({cut, last, d});
    }
    act = nx;
  }
  std::vector<R> out(n);
  for (int i = 0; i < n; i++) {
    if (heap[i]) { out[i] = a[i]; continue; }
    int s = i; while (!head[s]) s--;
    int e = i + 1; while (!head[e]) e++;
    int rank = 0;
    for (int j = s; j < e; j++) rank += a[j].key < a[i].key || (a[j].key == a[i].key && j < i);
    out[s + rank] = a[i];
  }
  a = out;
}
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
  // the level-parallel formulas of the device's voxel sort (cg_kernels.hip pcl_sort): cut =
  // L_0 or min(L_s, R_{s-1}), swaps (L_k, R_k) for k < s, stable sort inside the final ranges
  for (int it = 0; it < 20000; it++) {
    int n = (it % 7 == 0) ? (int)(rng() % 5000) : (int)(rng() % 400);
    unsigned kr = 1 + (unsigned)(rng() % ((it % 3 == 0) ? 3 : (it % 3 == 1) ? 50 : 100000));
    std::vector<R> a(n);
    for (int i = 0; i < n; i++) a[i] = {(unsigned)(rng() % kr), (unsigned)i};
    if (it % 11 == 0) std::sort(a.begin(), a.end(), [](const R& p, const R& q) { return p.key < q.key; });
    if (it % 13 == 0) std::reverse(a.begin(), a.end());
    for (int i = 0; i < n; i++) a[i].id = i;
    auto b = a;
    std::sort(a.begin(), a.end(), [](const R& p, const R& q) { return p.key < q.key; });
    levels_sort(b);
    for (int i = 0; i < n; i++) if (a[i].id != b[i].id) { bad++; break; }
  }
  if (bad) { printf("level model mismatches %ld\n", bad); return 5; }
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
