// Probe of the cluster-order sort (cg_sort.h): the ballot-scan wave sort (cg_std_sort_wave32)
// against the sequential restatement (cg_std_sort, one lane over LDS) on random tie-heavy
// inputs of n = 2..64 (one wave per case), and the cycles of both on 36 records (s_memrealtime).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I cones_perception_amd/csrc tools/sort_probe.hip -o tools/sort_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "cg_math.h"
#include "cg_sort.h"

__global__ void check(const uint32_t* sizes, const int* ns, uint32_t* bad, unsigned long long* t) {
    __shared__ uint64_t rec[64];
    __shared__ int32_t stk[3 * CG_SORT_STACK];
    const int l = threadIdx.x, c = blockIdx.x, n = ns[c];
    const uint32_t* sz = sizes + 64 * c;
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t r = l < n ? (sz[l] << 16) | (uint32_t)l : 0u;
    cg_std_sort_wave32(r, n);
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (l < n) rec[l] = ((uint64_t)sz[l] << 32) | (uint32_t)l;
    __syncthreads();
    unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
    if (l == 0) cg_std_sort(rec, (long)n, [](uint64_t a, uint64_t b) { return (a >> 32) < (b >> 32); }, stk);
    __syncthreads();
    unsigned long long t3 = __builtin_amdgcn_s_memrealtime();
    if (l < n && (r & 0xffffu) != (uint32_t)rec[l]) atomicAdd(bad, 1u);
    if (l == 0) { t[2 * c] = t1 - t0; t[2 * c + 1] = t3 - t2; }
}

int main() {
    const int cases = 4096;
    uint32_t* hs = (uint32_t*)calloc(64 * cases, 4);
    int* hn = (int*)calloc(cases, 4);
    srand(7);
    for (int c = 0; c < cases; c++) {
        hn[c] = c == 0 ? 36 : 2 + rand() % 63;
        const int range = 1 + rand() % (c % 3 == 0 ? 3 : (c % 3 == 1 ? 10 : 500));
        for (int i = 0; i < hn[c]; i++) hs[64 * c + i] = 2 + rand() % range;
    }
    uint32_t *ds, *dbad;
    int* dn;
    unsigned long long* dt;
    hipMalloc(&ds, 64 * cases * 4); hipMalloc(&dn, cases * 4); hipMalloc(&dbad, 4); hipMalloc(&dt, cases * 16);
    hipMemcpy(ds, hs, 64 * cases * 4, hipMemcpyHostToDevice);
    hipMemcpy(dn, hn, cases * 4, hipMemcpyHostToDevice);
    hipMemset(dbad, 0, 4);
    hipLaunchKernelGGL(check, dim3(cases), dim3(64), 0, 0, ds, dn, dbad, dt);
    uint32_t bad = 0;
    unsigned long long* t = (unsigned long long*)calloc(cases * 2, 8);
    hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost);
    hipMemcpy(t, dt, cases * 16, hipMemcpyDeviceToHost);
    std::printf("%d cases (n = 2..64, tie-heavy): %u elements placed differently\n", cases, bad);
    std::printf("first case (n = 36, cold caches): wave ballot sort %.2f us, one lane over LDS %.2f us\n", t[0] / 100.0,
                t[1] / 100.0);
    double a = 0, b = 0;
    int k = 0;
    for (int c = 1; c < cases; c++)
        if (hn[c] >= 30 && hn[c] <= 42) { a += t[2 * c]; b += t[2 * c + 1]; k++; }
    std::printf("mean over %d warm cases with n = 30..42: wave ballot sort %.2f us, one lane over LDS %.2f us\n", k,
                a / k / 100.0, b / k / 100.0);
    return bad != 0;
}
