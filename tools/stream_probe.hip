// stream_probe.hip — HBM read ceiling for the frame-streaming access pattern of pass 1
// (diagnostic, not part of the product). Each variant reads a batch of 64k-point xyzi frames
// (16 B per point) and reduces to one word per workgroup so the loads cannot be elided:
//   frame_x3 : one 512-lane workgroup per frame, global_load_dwordx3 per point (pass 1's shape)
//   frame_x4 : same, global_load_dwordx4
//   frame_x4_256 : 256-lane workgroups, two per frame half
//   flat_x4  : grid-stride dwordx4 over the whole batch, 4096 workgroups (the "ideal" stream)
// Prints GB/s per variant for 1 and 3 concurrently launched batches (3 streams).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int NPTS = 65536;

template <int BLOCK, int G>
__global__ __launch_bounds__(BLOCK) void frame_x3(const float* in, float* out, int parts) {
    const int f = blockIdx.x / parts, part = blockIdx.x % parts;
    const int per = NPTS / parts;
    const float* fb = in + (size_t)f * NPTS * 4 + (size_t)part * per * 4;
    float acc = 0.f;
    for (int k = 0; k < per / BLOCK; k += G) {
        float3 v[G];
#pragma unroll
        for (int j = 0; j < G; j++) v[j] = *(const float3*)(fb + ((size_t)(k + j) * BLOCK + threadIdx.x) * 4);
#pragma unroll
        for (int j = 0; j < G; j++) acc += v[j].x * v[j].y + v[j].z;
    }
    if (acc == 1234.5f) out[blockIdx.x] = acc;
}

template <int BLOCK, int G>
__global__ __launch_bounds__(BLOCK) void frame_x4(const float* in, float* out, int parts) {
    const int f = blockIdx.x / parts, part = blockIdx.x % parts;
    const int per = NPTS / parts;
    const float* fb = in + (size_t)f * NPTS * 4 + (size_t)part * per * 4;
    float acc = 0.f;
    for (int k = 0; k < per / BLOCK; k += G) {
        float4 v[G];
#pragma unroll
        for (int j = 0; j < G; j++) v[j] = *(const float4*)(fb + ((size_t)(k + j) * BLOCK + threadIdx.x) * 4);
#pragma unroll
        for (int j = 0; j < G; j++) acc += v[j].x * v[j].y + v[j].z + v[j].w;
    }
    if (acc == 1234.5f) out[blockIdx.x] = acc;
}

// pass-1-like: dwordx3 loads, A/B double buffer, ~WORK dependent VALU ops per point,
// dynamic LDS to pin occupancy (launch arg)
template <int BLOCK, int G, int WORK>
__global__ __launch_bounds__(BLOCK) void frame_work(const float* in, float* out, int parts) {
    extern __shared__ float lds[];
    const int f = blockIdx.x;
    const float* fb = in + (size_t)f * NPTS * 4;
    float acc = 0.f;
    float3 A[G], B[G];
    auto ld = [&](float3* v, int k) {
#pragma unroll
        for (int j = 0; j < G; j++) v[j] = *(const float3*)(fb + ((size_t)(k * G + j) * BLOCK + threadIdx.x) * 4);
    };
    auto work = [&](const float3* v) {
#pragma unroll
        for (int j = 0; j < G; j++) {
            float a = v[j].x, b = v[j].y, c = v[j].z;
#pragma unroll
            for (int w = 0; w < WORK / 3; w++) { a = fmaf(a, b, c); b = fmaf(b, c, a); c = fmaf(c, a, b); }
            acc += a + b + c;
        }
    };
    constexpr int NG = NPTS / BLOCK / G;
    ld(A, 0);
    for (int g = 0; g < NG; g += 2) {
        ld(B, g + 1);
        work(A);
        if (g + 2 < NG) ld(A, g + 2);
        work(B);
    }
    if (acc == 1234.5f) { lds[threadIdx.x] = acc; out[blockIdx.x] = lds[(threadIdx.x + 1) % BLOCK]; }
}

__global__ __launch_bounds__(256) void flat_x4(const float4* in, float* out, size_t n4) {
    float acc = 0.f;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        const float4 v = in[i];
        acc += v.x * v.y + v.z + v.w;
    }
    if (acc == 1234.5f) out[blockIdx.x] = acc;
}

int main(int argc, char** argv) {
    const int F = argc > 1 ? atoi(argv[1]) : 256;
    const int NB = 3;
    std::vector<float*> bufs(NB);
    for (int b = 0; b < NB; b++) {
        CHECK(hipMalloc(&bufs[b], (size_t)F * NPTS * 16));
        CHECK(hipMemset(bufs[b], 0, (size_t)F * NPTS * 16));
    }
    float* out;
    CHECK(hipMalloc(&out, 1 << 20));
    hipStream_t st[NB];
    for (int b = 0; b < NB; b++) CHECK(hipStreamCreateWithFlags(&st[b], hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const double bytes = (double)F * NPTS * 16;

    auto run = [&](const char* name, auto launch) {
        for (int conc : {1, 3}) {
            for (int w = 0; w < 3; w++) for (int b = 0; b < conc; b++) launch(bufs[b], st[b]);
            CHECK(hipDeviceSynchronize());
            const int reps = 20;
            CHECK(hipEventRecord(e0, 0));
            CHECK(hipDeviceSynchronize());
            for (int r = 0; r < reps; r++) for (int b = 0; b < conc; b++) launch(bufs[b], st[b]);
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            printf("%-22s streams=%d  %8.1f GB/s  (%.1f us per batch)\n", name, conc,
                   bytes * reps * conc / (ms * 1e-3) / 1e9, ms * 1e3 / (reps * conc));
        }
    };
    run("frame_x3 512 G8", [&](float* in, hipStream_t s) { hipLaunchKernelGGL((frame_x3<512, 8>), dim3(F), dim3(512), 0, s, in, out, 1); });
    run("frame_x3 512 G16", [&](float* in, hipStream_t s) { hipLaunchKernelGGL((frame_x3<512, 16>), dim3(F), dim3(512), 0, s, in, out, 1); });
    run("frame_x4 512 G8", [&](float* in, hipStream_t s) { hipLaunchKernelGGL((frame_x4<512, 8>), dim3(F), dim3(512), 0, s, in, out, 1); });
    run("frame_x4 512 G16", [&](float* in, hipStream_t s) { hipLaunchKernelGGL((frame_x4<512, 16>), dim3(F), dim3(512), 0, s, in, out, 1); });
    run("frame_x4 1024 G8", [&](float* in, hipStream_t s) { hipLaunchKernelGGL((frame_x4<1024, 8>), dim3(F), dim3(1024), 0, s, in, out, 1); });
    run("frame_x4 256x2 G8", [&](float* in, hipStream_t s) { hipLaunchKernelGGL((frame_x4<256, 8>), dim3(F * 2), dim3(256), 0, s, in, out, 2); });
    run("frame_x4 256x4 G8", [&](float* in, hipStream_t s) { hipLaunchKernelGGL((frame_x4<256, 8>), dim3(F * 4), dim3(256), 0, s, in, out, 4); });
    run("flat_x4 4096 wg", [&](float* in, hipStream_t s) { hipLaunchKernelGGL(flat_x4, dim3(4096), dim3(256), 0, s, (const float4*)in, out, (size_t)F * NPTS); });
    run("flat_x4 16384 wg", [&](float* in, hipStream_t s) { hipLaunchKernelGGL(flat_x4, dim3(16384), dim3(256), 0, s, (const float4*)in, out, (size_t)F * NPTS); });
    for (int lds_kb : {0, 60, 78}) {
        char nm[64];
        snprintf(nm, sizeof nm, "work0 lds%d", lds_kb);
        run(nm, [&](float* in, hipStream_t s) { hipLaunchKernelGGL((frame_work<512, 8, 0>), dim3(F), dim3(512), lds_kb * 1024, s, in, out, 1); });
        snprintf(nm, sizeof nm, "work60 lds%d", lds_kb);
        run(nm, [&](float* in, hipStream_t s) { hipLaunchKernelGGL((frame_work<512, 8, 60>), dim3(F), dim3(512), lds_kb * 1024, s, in, out, 1); });
        snprintf(nm, sizeof nm, "work120 lds%d", lds_kb);
        run(nm, [&](float* in, hipStream_t s) { hipLaunchKernelGGL((frame_work<512, 8, 120>), dim3(F), dim3(512), lds_kb * 1024, s, in, out, 1); });
    }
    return 0;
}
