// Timing probe of pcl_sort (cg_pcl.h) in one workgroup from LDS, with phase stamps
// (CG_PCL_PROBE), checked against std::sort on the host:  pcl_probe <n> <key range>
#define CG_PCL_PROBE 1
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include "../cones_perception_amd/csrc/cg_pcl.h"

#define NMAX 2048
__global__ __launch_bounds__(CG_BLOCK) void probe(const uint64_t* in, uint64_t* out, uint32_t n) {
    __shared__ __attribute__((aligned(16))) uint64_t E[NMAX], K[NMAX];
    __shared__ uint32_t w0[7 * (NMAX + 4)];
    __shared__ uint32_t red[8 * WAVES];
    for (uint32_t i = threadIdx.x; i < n; i += CG_BLOCK) E[i] = in[i];
    if (threadIdx.x == 0) g_pcl_probe_n = 0;
    __syncthreads();
    Work W{};
    W.KEY = K;
    W.A = w0; W.PAR = w0 + (NMAX + 4); W.CNT = w0 + 2 * (NMAX + 4); W.UK = w0 + 3 * (NMAX + 4);
    W.ORD = w0 + 4 * (NMAX + 4); W.LAB = (int32_t*)(w0 + 5 * (NMAX + 4)); W.OFF = w0 + 6 * (NMAX + 4);
    PCL_STAMP();
    pcl_sort(W, E, n, red);
    for (uint32_t i = threadIdx.x; i < n; i += CG_BLOCK) out[i] = K[i];
}
int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 230, kr = argc > 2 ? atoi(argv[2]) : 100;
    std::mt19937 rng(7);
    std::vector<uint64_t> h(n), o(n);
    for (uint32_t i = 0; i < n; i++) h[i] = ((uint64_t)(rng() % kr) << 32) | i;
    uint64_t *din, *dout;
    hipMalloc(&din, n * 8); hipMalloc(&dout, n * 8);
    hipMemcpy(din, h.data(), n * 8, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; rep++) hipLaunchKernelGGL(probe, dim3(1), dim3(CG_BLOCK), 0, 0, din, dout, n);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
    unsigned long long st[64]; unsigned int ns;
    hipMemcpyFromSymbol(st, HIP_SYMBOL(g_pcl_probe), sizeof(st));
    hipMemcpyFromSymbol(&ns, HIP_SYMBOL(g_pcl_probe_n), 4);
    hipMemcpy(o.data(), dout, n * 8, hipMemcpyDeviceToHost);
    std::vector<uint64_t> r = h;
    std::sort(r.begin(), r.end(), [](uint64_t a, uint64_t b) { return (a >> 32) < (b >> 32); });
    printf("n %u keys %u: %s; stamps (us):", n, kr, o == r ? "matches std::sort" : "MISMATCH");
    for (unsigned i = 1; i < ns; i++) printf(" %.2f", (st[i] - st[i - 1]) / 100.0);
    printf("  total %.2f\n", (st[ns - 1] - st[0]) / 100.0);
    return o == r ? 0 : 2;
}
