// isa_probe.hip — measured semantics of single instructions the kernels rely on (diagnostic).
//   cvt_pk_u8: v_cvt_pk_u8_f32 rounding, saturation and NaN handling
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>

__global__ void k_cvt(const float* in, unsigned* out, int n) {
    int i = threadIdx.x;
    if (i < n) {
        out[i] = __builtin_amdgcn_cvt_pk_u8_f32(in[i], 0u, 0u);
        out[n + i] = __builtin_amdgcn_cvt_pk_u8_f32(in[i], 2u, 0x11223344u);
    }
}

int main() {
    const float v[] = {NAN, -NAN, INFINITY, -INFINITY, -1.0f, -0.0f, 0.0f, 1e-40f, 0.4f, 0.5f, 0.6f, 1.5f, 2.5f,
                       3.5f, 254.4f, 254.5f, 254.6f, 255.0f, 255.4f, 255.5f, 255.6f, 256.0f, 300.0f, 1e9f,
                       -0.5f, -0.6f, 127.5f, 128.5f};
    const int n = sizeof v / sizeof v[0];
    float* d; unsigned* o;
    hipMalloc(&d, sizeof v); hipMalloc(&o, 2 * n * 4);
    hipMemcpy(d, v, sizeof v, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_cvt, dim3(1), dim3(64), 0, 0, d, o, n);
    unsigned h[2 * 64];
    hipMemcpy(h, o, 2 * n * 4, hipMemcpyDeviceToHost);
    for (int i = 0; i < n; i++) {
        unsigned b; memcpy(&b, &v[i], 4);
        printf("cvt_pk_u8 %-12g (0x%08x) -> %3u   byte2 into 0x11223344 -> 0x%08x\n", v[i], b, h[i], h[n + i]);
    }
    return 0;
}
