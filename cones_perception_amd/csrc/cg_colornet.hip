// cg_colornet.hip — the colour classifier service on the GPU:
// ColorClassifier.handle_classify_color / to_image (scripts/color_classifier_server.py:81-156)
// and the dam_net CNN it invokes through TFLite (models/dam_net/dam_net.tflite).
//
// One 256-lane workgroup per cone cloud:
//   to_image (color_classifier_server.py:131-156), in float64 as numpy computes it:
//     row = rint(-0.5 * (deg(atan2(z, sqrt(x*x + y*y))) + 15)), negative rows wrap (numpy
//     indexing), rows outside [-15, 14] raise IndexError in the reference;
//     col = rint(11 / ((hmax - hmin) + 1e-16) * (h - hmin)), h = deg(atan2(y, x));
//     pixel = (uint8) intensity (interp1d([0,255],[0,255]) is the identity on [0, 255] and raises
//     outside it); the last point of a pixel wins (numpy fancy assignment in order);
//   dam_net in float32 (layout of the .tflite graph):
//     CONV_2D 3x3x1->16 VALID + ReLU (13x10), MAX_POOL 2x2/2 (6x5), CONV_2D 3x3x16->32 VALID +
//     ReLU (4x3), MAX_POOL 2x2/2 (2x1), MUL, ADD (folded batch norm), RESHAPE (NHWC order),
//     FULLY_CONNECTED 64->3, SOFTMAX;
//   decision (color_classifier_server.py:112-116): max(p) >= 0.8 (as double) -> argmax + 1,
//   else 0 ("unknown").
// The network is 74k multiply-adds per cone and latency-bound at any batch a node produces:
// VALU in LDS, no MFMA (a 12 x 144 x 32 contraction per cone is below one MFMA tile pass).
#include <hip/hip_runtime.h>
#include <math.h>
#include "cg_internal.h"
#include "../../include/cones_gpu.h"

namespace {
constexpr int ROWS = 15, COLS = 12;
constexpr int C1H = 13, C1W = 10, C1C = 16;    // conv 1 output
constexpr int P1H = 6, P1W = 5;                // pool 1 output
constexpr int C2H = 4, C2W = 3, C2C = 32;      // conv 2 output
constexpr int P2H = 2, P2W = 1;                // pool 2 output
constexpr int FLAT = P2H * P2W * C2C;          // 64
constexpr int NCLS = 3;
// packed weights (include/cones_gpu.h CG_COLORNET_WEIGHTS)
constexpr int W1 = 0, B1 = W1 + C1C * 9, W2 = B1 + C1C, B2 = W2 + C2C * 9 * C1C, BNM = B2 + C2C, BNA = BNM + C2C,
              WD = BNA + C2C, BD = WD + NCLS * FLAT, WTOT = BD + NCLS;
static_assert(WTOT == CG_COLORNET_WEIGHTS, "packed colornet layout");
constexpr double RAD2DEG = 180.0 / 3.141592653589793;   // numpy rad2deg: x * (180.0 / NPY_PI)
}  // namespace

__global__ __launch_bounds__(256) void cg_colornet_kernel(const float4* pts, const uint32_t* offs, const float* w,
                                                          int32_t* colors, float* probs, uint8_t* images) {
    __shared__ float wl[WTOT];
    __shared__ int32_t owner[ROWS * COLS];
    __shared__ float img[ROWS * COLS];
    __shared__ float c1[C1H * C1W * C1C];
    __shared__ float p1[P1H * P1W * C1C];
    __shared__ float c2[C2H * C2W * C2C];
    __shared__ float flat[FLAT];
    __shared__ double red[2][256 / 64];
    __shared__ int bad[2];
    const uint32_t cone = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t s = offs[cone], e = offs[cone + 1], n = e - s;
    for (int i = tid; i < WTOT; i += 256) wl[i] = w[i];
    for (int i = tid; i < ROWS * COLS; i += 256) owner[i] = -1;
    if (tid < 2) bad[tid] = 0;
    if (n == 0) {   // the reference skips empty clouds (no entry in its response)
        if (tid == 0) colors[cone] = CG_COLOR_SKIPPED;
        if (tid < NCLS && probs) probs[cone * NCLS + tid] = 0.f;
        return;
    }
    // horizontal angle range
    double hmn = INFINITY, hmx = -INFINITY;
    for (uint32_t j = tid; j < n; j += 256) {
        const float4 p = pts[s + j];
        const double h = atan2((double)p.y, (double)p.x) * RAD2DEG;
        hmn = fmin(hmn, h);
        hmx = fmax(hmx, h);
    }
    for (int o = 32; o > 0; o >>= 1) {
        hmn = fmin(hmn, __shfl_xor(hmn, o));
        hmx = fmax(hmx, __shfl_xor(hmx, o));
    }
    if (lane == 0) { red[0][wv] = hmn; red[1][wv] = hmx; }
    __syncthreads();
    hmn = fmin(fmin(red[0][0], red[0][1]), fmin(red[0][2], red[0][3]));
    hmx = fmax(fmax(red[1][0], red[1][1]), fmax(red[1][2], red[1][3]));
    const double slope_h = (double)(COLS - 1) / ((hmx - hmn) + 1e-16);
    // pixel of each point; the last point of a pixel owns it
    for (uint32_t j = tid; j < n; j += 256) {
        const float4 p = pts[s + j];
        const double x = p.x, y = p.y, z = p.z;
        const double v = atan2(z, sqrt(x * x + y * y)) * RAD2DEG;
        const double r = rint(-0.5 * (v - (-15.0)));
        const double c = rint(slope_h * (atan2(y, x) * RAD2DEG - hmn));
        if (!(r >= -ROWS && r < ROWS) || !(c >= 0.0 && c < COLS)) { bad[0] = 1; continue; }
        if (!((double)p.w >= 0.0 && (double)p.w <= 255.0)) bad[1] = 1;
        const int row = (int)r < 0 ? (int)r + ROWS : (int)r;
        atomicMax(&owner[row * COLS + (int)c], (int32_t)j);
    }
    __syncthreads();
    for (int i = tid; i < ROWS * COLS; i += 256) {
        const int j = owner[i];
        // float64 -> uint8 truncates (numpy's C cast); a NaN intensity is stored as 0
        const double iv = j >= 0 ? (double)pts[s + j].w : 0.0;
        img[i] = (iv >= 0.0 && iv < 256.0) ? (float)(uint32_t)iv : 0.f;
        if (images) images[(size_t)cone * ROWS * COLS + i] = (uint8_t)img[i];
    }
    __syncthreads();
    // conv 1 + ReLU: out (y, x, o), NHWC
    for (int i = tid; i < C1H * C1W * C1C; i += 256) {
        const int o = i % C1C, xy = i / C1C, x = xy % C1W, y = xy / C1W;
        float acc = 0.f;
        for (int ky = 0; ky < 3; ky++)
            for (int kx = 0; kx < 3; kx++) acc += img[(y + ky) * COLS + (x + kx)] * wl[W1 + o * 9 + ky * 3 + kx];
        c1[i] = fmaxf(acc + wl[B1 + o], 0.f);
    }
    __syncthreads();
    for (int i = tid; i < P1H * P1W * C1C; i += 256) {
        const int o = i % C1C, xy = i / C1C, x = xy % P1W, y = xy / P1W;
        const float* q = c1 + ((2 * y) * C1W + 2 * x) * C1C + o;
        p1[i] = fmaxf(fmaxf(q[0], q[C1C]), fmaxf(q[C1W * C1C], q[C1W * C1C + C1C]));
    }
    __syncthreads();
    // conv 2 + ReLU
    for (int i = tid; i < C2H * C2W * C2C; i += 256) {
        const int o = i % C2C, xy = i / C2C, x = xy % C2W, y = xy / C2W;
        float acc = 0.f;
        for (int ky = 0; ky < 3; ky++)
            for (int kx = 0; kx < 3; kx++) {
                const float* a = p1 + ((y + ky) * P1W + (x + kx)) * C1C;
                const float* b = wl + W2 + ((o * 3 + ky) * 3 + kx) * C1C;
                for (int c = 0; c < C1C; c++) acc += a[c] * b[c];
            }
        c2[i] = fmaxf(acc + wl[B2 + o], 0.f);
    }
    __syncthreads();
    // pool 2, batch-norm MUL then ADD (two roundings, as two graph ops), flatten (h, w, c)
    if (tid < FLAT) {
        const int o = tid % C2C, y = tid / C2C;
        const float* q = c2 + ((2 * y) * C2W) * C2C + o;
        const float m = fmaxf(fmaxf(q[0], q[C2C]), fmaxf(q[C2W * C2C], q[C2W * C2C + C2C]));
        const float t = m * wl[BNM + o];
        flat[tid] = t + wl[BNA + o];
    }
    __syncthreads();
    if (tid == 0) {
        float lg[NCLS];
        for (int k = 0; k < NCLS; k++) {
            float acc = 0.f;
            for (int i = 0; i < FLAT; i++) acc += flat[i] * wl[WD + k * FLAT + i];
            lg[k] = acc + wl[BD + k];
        }
        const float mx = fmaxf(fmaxf(lg[0], lg[1]), lg[2]);
        float ex[NCLS], sum = 0.f;
        for (int k = 0; k < NCLS; k++) { ex[k] = expf(lg[k] - mx); sum += ex[k]; }
        float pr[NCLS];
        int best = 0;
        for (int k = 0; k < NCLS; k++) {
            pr[k] = ex[k] / sum;
            if (probs) probs[cone * NCLS + k] = pr[k];
            if (pr[k] > pr[best]) best = k;
        }
        int col = (double)pr[best] >= 0.8 ? best + 1 : 0;
        // the reference evaluates interp1d (ValueError) before the indexed assignment (IndexError)
        if (bad[1]) col = CG_COLOR_RANGE_ERROR;
        else if (bad[0]) col = CG_COLOR_INDEX_ERROR;
        colors[cone] = col;
    }
}

int cg_launch_colornet(const float4* pts, const uint32_t* offs, uint32_t n_cones, const float* w, int32_t* colors,
                       float* probs, uint8_t* images, hipStream_t s) {
    if (n_cones)
        hipLaunchKernelGGL(cg_colornet_kernel, dim3(n_cones), dim3(256), 0, s, pts, offs, w, colors, probs, images);
    return hipGetLastError();
}
