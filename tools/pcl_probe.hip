// pcl_sort (cg_pcl.h) on the device against std::sort on the host: many random cases (n up to
// 2048, tie-heavy and distinct keys, sorted / reversed / organ-pipe inputs), one workgroup per
// case from LDS, plus phase stamps (CG_PCL_PROBE) of one case:  pcl_probe [cases] [stamp n]
// Every seventh case starts with a small depth budget (0-3), checked against libstdc++'s own
// __introsort_loop + __final_insertion_sort with that budget, so heapsort fallbacks run.
#define CG_PCL_PROBE 1
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include "../cones_perception_amd/csrc/cg_pcl.h"

#define NMAX 2048
__global__ __launch_bounds__(CG_BLOCK) void probe(const uint64_t* in, uint64_t* out, const uint32_t* offs, const int* depth, int stamp) {
    __shared__ __attribute__((aligned(16))) uint64_t E[NMAX], K[NMAX], E2[NMAX];
    __shared__ uint32_t w0[7 * (NMAX + 4)];
    __shared__ uint32_t red[8 * WAVES];
    const uint32_t o = offs[blockIdx.x], n = offs[blockIdx.x + 1] - o;
    for (uint32_t i = threadIdx.x; i < n; i += CG_BLOCK) E[i] = in[o + i];
    if (stamp && threadIdx.x == 0) g_pcl_probe_n = 0;
    __syncthreads();
    Work W{};
    W.KEY = K;
    W.A = w0; W.PAR = w0 + (NMAX + 4); W.CNT = w0 + 2 * (NMAX + 4); W.UK = w0 + 3 * (NMAX + 4);
    W.ORD = w0 + 4 * (NMAX + 4); W.LAB = (int32_t*)(w0 + 5 * (NMAX + 4)); W.OFF = w0 + 6 * (NMAX + 4);
    if (stamp) PCL_STAMP();
    pcl_sort<4, true>(W, E, n, red, depth[blockIdx.x], E2);
    for (uint32_t i = threadIdx.x; i < n; i += CG_BLOCK) out[o + i] = K[i];
}
int main(int argc, char** argv) {
    const int cases = argc > 1 ? atoi(argv[1]) : 4000;
    const uint32_t sn = argc > 2 ? atoi(argv[2]) : 243;
    std::mt19937_64 rng(7);
    std::vector<uint64_t> h;
    std::vector<uint32_t> offs{0};
    std::vector<int> dep;
    for (int c = 0; c < cases; c++) {
        const uint32_t n = c == 0 ? sn : (c % 5 == 0) ? (uint32_t)(rng() % (NMAX + 1)) : (uint32_t)(rng() % 600);
        const uint32_t kr = 1 + (uint32_t)(rng() % ((c % 3 == 0) ? 4 : (c % 3 == 1) ? 60 : 100000));
        std::vector<uint32_t> k(n);
        for (uint32_t i = 0; i < n; i++) k[i] = (uint32_t)(rng() % kr);
        if (c % 11 == 1) std::sort(k.begin(), k.end());
        if (c % 13 == 2) std::sort(k.rbegin(), k.rend());
        if (c % 17 == 3) for (uint32_t i = 0; i < n; i++) k[i] = std::min(i, n - i);   // organ pipe
        for (uint32_t i = 0; i < n; i++) h.push_back(((uint64_t)k[i] << 32) | i);
        offs.push_back((uint32_t)h.size());
        dep.push_back(c % 7 == 4 ? (int)(rng() % 4) : -1);
    }
    std::vector<uint64_t> o(h.size());
    uint64_t *din, *dout;
    uint32_t* doff;
    int* ddep;
    hipMalloc(&din, h.size() * 8 + 8); hipMalloc(&dout, h.size() * 8 + 8); hipMalloc(&doff, offs.size() * 4);
    hipMalloc(&ddep, dep.size() * 4);
    hipMemcpy(ddep, dep.data(), dep.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(din, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(doff, offs.data(), offs.size() * 4, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; rep++) hipLaunchKernelGGL(probe, dim3(1), dim3(CG_BLOCK), 0, 0, din, dout, doff, ddep, 1);
    if (hipDeviceSynchronize() != hipSuccess) { printf("stamp launch failed\n"); return 1; }
    unsigned long long st[64]; unsigned int ns;
    hipMemcpyFromSymbol(st, HIP_SYMBOL(g_pcl_probe), sizeof(st));
    hipMemcpyFromSymbol(&ns, HIP_SYMBOL(g_pcl_probe_n), 4);
    ns = ns < 64 ? ns : 64;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(probe, dim3(cases), dim3(CG_BLOCK), 0, 0, din, dout, doff, ddep, 0);
    hipEventRecord(e1, 0);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(o.data(), dout, h.size() * 8, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int c = 0; c < cases; c++) {
        std::vector<uint64_t> r(h.begin() + offs[c], h.begin() + offs[c + 1]);
        auto less = [](uint64_t a, uint64_t b) { return (a >> 32) < (b >> 32); };
        if (dep[c] < 0 || r.empty()) {
            std::sort(r.begin(), r.end(), less);
        } else {
            auto cmp = __gnu_cxx::__ops::__iter_comp_iter(less);
            std::__introsort_loop(r.begin(), r.end(), (long)dep[c], cmp);
            std::__final_insertion_sort(r.begin(), r.end(), cmp);
        }
        if (!std::equal(r.begin(), r.end(), o.begin() + offs[c])) {
            if (bad < 5) printf("case %d (n %u) MISMATCH\n", c, offs[c + 1] - offs[c]);
            bad++;
        }
    }
    printf("%d cases, %d mismatches; all cases %.3f ms; case 0 (n %u) stamps (us):", cases, bad, ms, sn);
    for (unsigned i = 1; i < ns; i++) printf(" %.2f", (st[i] - st[i - 1]) / 100.0);
    printf("  total %.2f\n", (st[ns - 1] - st[0]) / 100.0);
    return bad ? 2 : 0;
}
