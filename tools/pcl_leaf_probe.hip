// pcl_block_sort (cg_pcl.h) in the large path's leaf configuration (lg_pcl_leaf: up to 4,096
// records in LDS, 8 per thread, scratch in LDS, results straight to global memory) against
// std::sort, with phase stamps (CG_PCL_PROBE) of case 0:
//   pcl_leaf_probe [cases] [stamp n] [keys per distinct key of case 0]
// Case 0 imitates a C5 leaf: n records, about n / tie distinct keys in random order. Every
// seventh case starts with a depth budget of 0-3, checked against libstdc++'s own
// __introsort_loop + __final_insertion_sort with that budget (heapsort fallbacks).
#define CG_PCL_PROBE 1
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include "../cones_perception_amd/csrc/cg_pcl.h"

#define LEAF 4096
#define LDSB (8 * LEAF + 4 * 4 * (LEAF + 4))
struct ProbeOut {
    uint64_t* o;
    __device__ __forceinline__ void operator()(uint32_t i, uint64_t r) const { o[i] = r; }
};
__global__ __launch_bounds__(CG_BLOCK) void probe(const uint64_t* in, uint64_t* out, const uint32_t* offs,
                                                  const int* depth, int stamp) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[LDSB];
    __shared__ uint32_t red[8 * WAVES];
    const uint32_t o = offs[blockIdx.x], n = offs[blockIdx.x + 1] - o;
    lds_u64* const El = (lds_u64*)(uint64_t*)smem;
    lds_u32* const w0 = (lds_u32*)(uint32_t*)(smem + 8 * LEAF);
    const PbScratch<PbLds> PS{w0, w0 + (LEAF + 4), w0 + 2 * (LEAF + 4), w0 + 3 * (LEAF + 4)};
    lds_u32* const Rl = (lds_u32*)red;
    for (uint32_t i = threadIdx.x; i < n; i += CG_BLOCK) El[i] = in[o + i];
    if (stamp && threadIdx.x == 0) g_pcl_probe_n = 0;
    __syncthreads();
    if (stamp) PCL_STAMP();
    const ProbeOut po{out + o};
    const uint32_t d = depth[blockIdx.x] >= 0 ? (uint32_t)depth[blockIdx.x] : (uint32_t)(2 * cg_lg((long)n));
    if (n <= CG_BLOCK) pcl_block_sort<1, PbLds>(El, po, n, d, PS, Rl);
    else if (n <= 2 * CG_BLOCK) pcl_block_sort<2, PbLds>(El, po, n, d, PS, Rl);
    else if (n <= 4 * CG_BLOCK) pcl_block_sort<4, PbLds>(El, po, n, d, PS, Rl);
    else pcl_block_sort<8, PbLds>(El, po, n, d, PS, Rl);
    if (stamp) PCL_STAMP();
}
int main(int argc, char** argv) {
    const int cases = argc > 1 ? atoi(argv[1]) : 400;
    const uint32_t sn = argc > 2 ? atoi(argv[2]) : 4096;
    const uint32_t tie = argc > 3 ? atoi(argv[3]) : 9;
    std::mt19937_64 rng(11);
    std::vector<uint64_t> h;
    std::vector<uint32_t> offs{0};
    std::vector<int> dep;
    for (int c = 0; c < cases; c++) {
        const uint32_t n = c == 0 ? sn : (uint32_t)(rng() % (LEAF + 1));
        const uint32_t kr = c == 0 ? std::max(1u, sn / tie) : 1 + (uint32_t)(rng() % ((c % 3 == 0) ? 8 : (c % 3 == 1) ? 600 : 100000));
        std::vector<uint32_t> k(n);
        for (uint32_t i = 0; i < n; i++) k[i] = (uint32_t)(rng() % kr);
        if (c % 11 == 1) std::sort(k.begin(), k.end());
        if (c % 13 == 2) std::sort(k.rbegin(), k.rend());
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
    printf("%d cases, %d mismatches; all cases %.3f ms; case 0 (n %u, %u per key) stamps (us):", cases, bad, ms, sn, tie);
    for (unsigned i = 1; i < ns; i++) printf(" %.2f", (st[i] - st[i - 1]) / 100.0);
    printf("  total %.2f (%u stamps)\n", (st[ns - 1] - st[0]) / 100.0, ns);
    return bad ? 2 : 0;
}
