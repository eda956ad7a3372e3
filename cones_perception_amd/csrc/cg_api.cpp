// cg_api.cpp — host side of the C-ABI (include/cones_gpu.h): handle, parameter preparation,
// staging, kernel launches and result download. No compute happens here: every per-point
// operation of the hot path runs in cg_kernels.hip. The host only (1) resolves the
// reference's parameter expressions into exact device thresholds once per cg_set_params,
// (2) copies PointCloud2 bytes in and results out.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <chrono>
#include <cstring>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <mutex>
#include <string>
#include <thread>
#include <vector>
#include <immintrin.h>
#include "../../include/cones_gpu_debug.h"
#include "cg_internal.h"
#include "cg_math.h"
#include "cg_host.h"

namespace {

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    const int rc = cg_vfail(code, fmt, ap);
    va_end(ap);
    return rc;
}

#define HIPCHK(expr)                                                                     \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            return fail(e_ == hipErrorOutOfMemory ? CG_E_OOM : CG_E_DEVICE, "%s: %s (%s:%d)", \
                        #expr, hipGetErrorString(e_), __FILE__, __LINE__);               \
    } while (0)

int prepare(const cg_params& p, CgDevParams& d) { return cg_prepare_params(p, d); }

}  // namespace

// Host helper threads for the single-frame staging copy (C2). The split launch's chunk
// workgroups each wait for their chunk of the message to be copied into pinned memory and
// published; one thread publishing 16 chunks of 64 KiB one after another took 15.5 us, and the
// GPU's PCIe reads of the last chunks waited for it (profiles/r5_c2_stamps.txt). The pool's
// threads copy and publish interleaved chunks beside the calling thread (chunk c by part
// c % parts; the caller is part 0), so every chunk is published within a few us of the launch.
// Between calls a helper spins for CG_STAGE_SPIN_US (the node's next frame usually comes within
// it when frames queue), then sleeps on a condition variable. CG_STAGE_THREADS sets the helper
// count (default 3; 0: the caller copies every chunk, as before).
struct StagePool {
    std::vector<std::thread> th;
    std::atomic<uint32_t> job{0};       // the current job's number (helpers start when it changes)
    std::atomic<uint32_t> left{0};      // helpers still copying the current job
    std::atomic<int> sleepers{0};
    std::atomic<bool> quit{false};
    std::mutex mu;
    std::condition_variable cv;
    uint64_t spin_ns = 2000000;
    // the current job (written before `job` is released)
    const uint8_t* src = nullptr;
    uint8_t* dst = nullptr;
    uint32_t* flags = nullptr;
    uint32_t seq = 0, n = 0, step = 0, nch = 0, parts = 1;
    bool copy = true;

    void chunks(uint32_t part) const {
        for (uint32_t c = part; c < nch; c += parts) {
            if (copy && (uint64_t)c * CG_SPLIT_CHUNK < n) {
                const size_t b0 = (size_t)c * CG_SPLIT_CHUNK * step;
                const size_t nb = (size_t)std::min<uint32_t>(CG_SPLIT_CHUNK, n - c * CG_SPLIT_CHUNK) * step;
                std::memcpy(dst + b0, src + b0, nb);
            }
            __atomic_thread_fence(__ATOMIC_SEQ_CST);   // also orders a memcpy's non-temporal stores
            __atomic_store_n(&flags[c], seq, __ATOMIC_RELEASE);
        }
    }
    void worker(uint32_t part) {
        uint32_t seen = 0;
        for (;;) {
            auto t0 = std::chrono::steady_clock::now();
            while (job.load(std::memory_order_acquire) == seen && !quit.load(std::memory_order_relaxed)) {
                _mm_pause();
                if ((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0)
                        .count() > spin_ns) {
                    std::unique_lock<std::mutex> lk(mu);
                    sleepers++;
                    cv.wait(lk, [&] { return job.load(std::memory_order_acquire) != seen || quit.load(); });
                    sleepers--;
                    t0 = std::chrono::steady_clock::now();
                }
            }
            if (quit.load()) return;
            seen = job.load(std::memory_order_acquire);
            chunks(part);
            left.fetch_sub(1, std::memory_order_release);
        }
    }
    ~StagePool() {
        {
            std::lock_guard<std::mutex> lk(mu);
            quit.store(true);
        }
        cv.notify_all();
        for (auto& t : th) t.join();
    }
};

struct cg_handle {
    int device = 0;
    cg_params params{};
    CgDevParams dp{};
    hipStream_t stream = nullptr;
    // batch result buffers
    uint32_t cap_frames = 0, cap_points = 0;
    uint32_t* d_hdr = nullptr;
    float4* d_vox = nullptr;
    int32_t* d_lab = nullptr;
    int32_t* d_offs = nullptr;
    int32_t* d_idx = nullptr;
    float2* d_cen = nullptr;
    uint8_t* d_ground = nullptr;
    uint8_t* d_scratch = nullptr;
    uint64_t scratch_stride = 0;
    // single-frame staging
    uint8_t* d_in = nullptr;
    size_t d_in_bytes = 0;
    uint8_t* h_stage = nullptr;   // pinned, coherent (split kernels read it while the host fills it)
    uint32_t* h_flags = nullptr;  // pinned, coherent: per-chunk publish words of the staging buffer
    uint32_t* h_flags_dev = nullptr;
    uint32_t stage_seq = 0;
    size_t h_stage_bytes = 0;
    StagePool* pool = nullptr;       // staging helper threads (created with the first split call)
    bool pool_tried = false;
    // last batch
    uint32_t last_frames = 0, last_points = 0;
    int last_mode = -1;
    hipStream_t last_stream = nullptr;
    // orders a batch call on another stream after the handle's previous work (its result and
    // scratch slots are reused): recorded on the previous stream at the switch
    hipEvent_t ev_switch = nullptr;
    // host results
    uint32_t h_hdr[CG_HDR_WORDS] = {};
    uint32_t* d_split = nullptr;     // split single-frame launch state (CG_SPLIT_WORDS)
    bool packed = false;             // the last single-frame launch left its results in d_pack
    uint32_t* d_pack = nullptr;      // fetch_frame: one frame's results packed (CG_PACK_WORDS)
    uint32_t* h_pack = nullptr;      // pinned copy of it; the results handed out point into it
    uint32_t* h_pack_dev = nullptr;  // h_pack's device address: the split launch packs straight into it
    std::vector<float> h_vox, h_cen;
    std::vector<int32_t> h_lab, h_offs, h_idx;
    uint8_t* h_ground = nullptr;  // pinned
    size_t h_ground_bytes = 0;
    // frames of more than CG_MAX_POINTS points (cg_large.hip): scratch for one frame
    uint8_t* d_large = nullptr;
    uint32_t* h_meta = nullptr;      // pinned: the large path's per-frame meta read
    uint32_t large_points = 0;
    // a second large-frame scratch set: batches of several large frames pipeline over two
    LgScratch lg2{};
    uint8_t* d_large2 = nullptr;
    uint32_t* h_meta2 = nullptr;
    uint32_t large2_points = 0;
    LgScratch lg{};
    LgGraphs* lg_graphs = nullptr;   // captured large frames (cg_run_large), for its scratch set
    uint32_t* h_hint = nullptr;      // pinned: the device-sized large path's level hint (LgScratch::hint)
    int route = 0;                // cg_debug_route
    uint32_t retries = 0;         // single-frame calls re-run by DMA after a staging timeout
    unsigned long long* next_span = nullptr;   // cg_debug_launch_spans: the next launch's span slot
    uint32_t spans_left = 0;                   //   and how many launches still record
    cg_tile tile{};               // the rank's tile (cg_tile_front .. cg_tile_decide)
    bool tile_ready = false;
    // the last single-frame call, for cg_recrop
    bool last_single = false;
    CgLaunch last_in{};
    // the last cg_run_batch, for cg_batch_recrop (its input stays the caller's device memory)
    CgLaunch last_batch{};
    int batch_kmode = 0;
    bool batch_valid = false;
    uint32_t pack_seq = 0;   // the last split launch's done word (CG_PACK_DONE)
    uint32_t last_k = 0;
    uint32_t* d_seckeys = nullptr;   // 18 words per frame inside d_hdr (not owned)
    RcBox* d_boxes = nullptr;
    uint32_t* d_rc_cnt = nullptr;    // boxes x blocks, twice (counts, offsets)
    size_t rc_cnt_cap = 0;
    float4* d_rc_out = nullptr;
    size_t rc_out_cap = 0;
    std::vector<uint32_t> h_rc_cnt, h_rc_off;
    std::vector<float> h_rc_pts, h_rc_dev;
    // colour classifier (cg_colornet_set / cg_classify_colors)
    float* d_cn_w = nullptr;
    float4* d_cn_pts = nullptr;
    size_t cn_pts_cap = 0;
    uint32_t* d_cn_offs = nullptr;   // offsets, then colors (int32), probs (float), images (bytes)
    size_t cn_cap = 0;
    // diagnostics
    bool stamps_on = false;
    uint64_t* d_stamps = nullptr;
    uint32_t stamps_frames = 0;
};

namespace {

// The handle's private stream, created lazily: batch calls that pass their own stream never
// need one, and every stream costs one of the process's few hardware queues.
int own_stream(cg_handle* h) {
    if (h->stream) return CG_OK;
    HIPCHK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    return CG_OK;
}

void free_batch(cg_handle* h) {
    (void)hipFree(h->d_hdr); (void)hipFree(h->d_vox); (void)hipFree(h->d_lab); (void)hipFree(h->d_offs);
    (void)hipFree(h->d_idx); (void)hipFree(h->d_cen); (void)hipFree(h->d_ground); (void)hipFree(h->d_scratch);
    h->d_hdr = nullptr; h->d_vox = nullptr; h->d_lab = nullptr; h->d_offs = nullptr;
    h->d_idx = nullptr; h->d_cen = nullptr; h->d_ground = nullptr; h->d_scratch = nullptr;
    h->d_seckeys = nullptr;
    h->cap_frames = h->cap_points = 0;
}

int ensure_batch(cg_handle* h, uint32_t frames, uint32_t points, bool ground) {
    // every caller writes (or reallocates) the per-frame result slots: cg_batch_recrop may
    // read them again only after the next cg_run_batch (which sets batch_valid afterwards)
    h->batch_valid = false;
    const uint32_t pts = std::max<uint32_t>(points, 1);
    const bool need_ground = ground && h->d_ground == nullptr;
    if (frames <= h->cap_frames && pts <= h->cap_points && !need_ground) return CG_OK;
    const uint32_t nf = std::max(frames, h->cap_frames), np = std::max(pts, h->cap_points);
    const bool had_ground = h->d_ground != nullptr || ground;
    free_batch(h);
    const uint64_t F = nf, C = np;
    // headers, then each frame's 18 final sector-minimum keys (cg_recrop of a pipeline frame)
    HIPCHK(hipMalloc(&h->d_hdr, F * (CG_HDR_WORDS + CG_NUM_BINS + 1) * 4));
    h->d_seckeys = h->d_hdr + F * CG_HDR_WORDS;
    HIPCHK(hipMalloc(&h->d_vox, F * C * 16));
    HIPCHK(hipMalloc(&h->d_lab, F * C * 4));
    HIPCHK(hipMalloc(&h->d_offs, F * (C + 1) * 4));
    HIPCHK(hipMalloc(&h->d_idx, F * C * 4));
    HIPCHK(hipMalloc(&h->d_cen, F * C * 8));
    // the frame kernel's HBM fallback (M > CG_MMAX) serves frames of <= CG_MAX_POINTS points
    h->scratch_stride = (cg_scratch_bytes(std::min<uint32_t>(np, CG_MAX_POINTS)) + 255) & ~255ull;
    HIPCHK(hipMalloc(&h->d_scratch, F * h->scratch_stride));
    if (had_ground) HIPCHK(hipMalloc(&h->d_ground, F * C * 32));
    h->cap_frames = nf;
    h->cap_points = np;
    return CG_OK;
}

int check_view(const cg_cloud_view* v) { return cg_check_view(v); }

// Stage a PointCloud2 data block as one contiguous device frame. Aligned, unpadded rows are
// uploaded verbatim; padded rows or unaligned fields are re-packed (pure byte moves, the
// memcpy half of pcl::fromROSMsg) to x,y,z,intensity at 0,4,8,12.
// defer (with zero_copy, verbatim layouts): the bytes are not copied here; the caller copies
// them after the launch with publish_chunks.
int stage_frame(cg_handle* h, const cg_cloud_view* v, CgLaunch& L, bool zero_copy = false, bool* deferred = nullptr) {
    const uint32_t n = v->width * v->height;
    const bool aligned = v->point_step % 4 == 0 && (v->off_x < 0 || v->off_x % 4 == 0) &&
                         (v->off_y < 0 || v->off_y % 4 == 0) && (v->off_z < 0 || v->off_z % 4 == 0) &&
                         (v->off_intensity < 0 || v->off_intensity % 4 == 0);
    const bool contiguous = v->height <= 1 || v->row_step == v->width * v->point_step;
    const bool verbatim = aligned && contiguous;
    const uint32_t step = verbatim ? v->point_step : 16;
    const size_t bytes = std::max<size_t>((size_t)n * step, 16);
    if (bytes > h->h_stage_bytes) {
        // (the publish words h_flags do not depend on the frame size: they live as long as the
        // handle; freeing them here with the staging buffer left the host and the already
        // launched chunk workgroups on an unmapped page, the round-3 fault)
        if (h->h_stage) (void)hipHostFree(h->h_stage);
        h->h_stage = nullptr;
        HIPCHK(hipHostMalloc(&h->h_stage, bytes, hipHostMallocCoherent));
        h->h_stage_bytes = bytes;
    }
    if (bytes > h->d_in_bytes) {
        if (h->d_in) (void)hipFree(h->d_in);
        h->d_in = nullptr;
        HIPCHK(hipMalloc(&h->d_in, bytes));
        h->d_in_bytes = bytes;
    }
    const uint8_t* src = (const uint8_t*)v->data;
    if (deferred) *deferred = zero_copy && verbatim && n;
    if (verbatim) {
        if (n && !(deferred && *deferred)) std::memcpy(h->h_stage, src, (size_t)n * step);
        L.point_step = v->point_step;
        L.off_x = v->off_x; L.off_y = v->off_y; L.off_z = v->off_z; L.off_i = v->off_intensity;
    } else {
        const int32_t offs[4] = {v->off_x, v->off_y, v->off_z, v->off_intensity};
        for (uint32_t r = 0; r < v->height; r++)
            for (uint32_t c = 0; c < v->width; c++) {
                const uint8_t* p = src + (size_t)r * v->row_step + (size_t)c * v->point_step;
                uint8_t* q = h->h_stage + ((size_t)r * v->width + c) * 16;
                for (int a = 0; a < 4; a++) {
                    if (offs[a] >= 0) std::memcpy(q + 4 * a, p + offs[a], 4);
                    else std::memset(q + 4 * a, 0, 4);
                }
            }
        L.point_step = 16;
        L.off_x = 0; L.off_y = 4; L.off_z = 8; L.off_i = 12;
    }
    // zero_copy (split single frames): the kernel's chunk workgroups read the pinned staging
    // buffer over PCIe and write the device copy themselves; no DMA, no DMA-to-kernel gap
    if (zero_copy) L.in_host = h->h_stage;
    else if (n) HIPCHK(hipMemcpyAsync(h->d_in, h->h_stage, (size_t)n * step, hipMemcpyHostToDevice, h->stream));
    L.in = h->d_in;
    L.frame_stride = (uint64_t)n * step;
    L.n_frames = 1;
    L.n_points = n;
    L.is_dense = v->is_dense;
    return CG_OK;
}

void fill_launch_outputs(cg_handle* h, CgLaunch& L) {
    L.cap = h->cap_points;
    L.hdr = h->d_hdr; L.vox = h->d_vox; L.lab = h->d_lab; L.offs = h->d_offs;
    L.idx = h->d_idx; L.cen = h->d_cen; L.ground = h->d_ground;
    L.scratch = h->d_scratch; L.scratch_stride = h->scratch_stride;
    L.stamps = nullptr;
    if (h->stamps_on) {
        // stamps are indexed by workgroup: a split single-frame launch has one workgroup per
        // chunk (up to CG_MAX_POINTS / CG_SPLIT_CHUNK), more than the handle's frame capacity
        const uint32_t need = std::max<uint32_t>(h->cap_frames, CG_MAX_POINTS / CG_SPLIT_CHUNK);
        if (h->stamps_frames < need) {
            (void)hipFree(h->d_stamps);
            h->d_stamps = nullptr;
            if (hipMalloc(&h->d_stamps, (size_t)need * 32 * 8) == hipSuccess)
                h->stamps_frames = need;
            else
                h->stamps_frames = 0;
        }
        if (h->d_stamps) (void)hipMemset(h->d_stamps, 0, (size_t)h->stamps_frames * 32 * 8);
        L.stamps = h->d_stamps;
    }
}

// The large-path scratch with the diagnostic route's settings applied: every entry point
// that runs the large backend takes its copy from here, so a route set (or cleared) by
// cg_debug_route reaches the tile and halo protocols too, whatever ran last.
LgScratch route_scratch(cg_handle* h, bool second = false) {
    LgScratch S = second ? h->lg2 : h->lg;
    S.force_global = (h->route == 2 || h->route == 5) ? 1u : 0u;
    S.pcl_levels_cap = h->route == 5 ? 1u : 0u;
    S.force_wait_fail = h->route == 10 ? 1u : 0u;
    return S;
}

int ensure_large(cg_handle* h, uint32_t n) {
    if (n <= h->large_points && h->d_large) return CG_OK;
    if (h->d_large) (void)hipFree(h->d_large);   // (waits for the device: no graph still runs)
    cg_large_graphs_free(h->lg_graphs);           // they name the old scratch
    h->lg_graphs = nullptr;
    h->d_large = nullptr;
    h->large_points = 0;
    HIPCHK(hipMalloc(&h->d_large, cg_large_bytes(n)));
    HIPCHK(hipMemset(h->d_large, 0, cg_large_bytes(n)));   // the scans' status words start zeroed
    cg_large_layout(h->d_large, n, h->lg);
    if (!h->h_meta) HIPCHK(hipHostMalloc((void**)&h->h_meta, LG_META_WORDS * 4, hipHostMallocDefault));
    h->lg.hmeta = h->h_meta;
    if (!h->h_hint) {
        HIPCHK(hipHostMalloc((void**)&h->h_hint, 64, hipHostMallocCoherent));
        std::memset(h->h_hint, 0, 64);
    }
    HIPCHK(hipHostGetDevicePointer((void**)&h->lg.hint, h->h_hint, 0));
    h->large_points = n;
    return CG_OK;
}

// Frames of <= CG_MAX_POINTS points run as one batch launch of the frame kernel; larger
// frames (or every frame, under cg_debug_route) go through the multi-workgroup large path.
int ensure_large2(cg_handle* h, uint32_t n) {
    if (n <= h->large2_points && h->d_large2) return CG_OK;
    if (h->d_large2) (void)hipFree(h->d_large2);
    h->d_large2 = nullptr;
    h->large2_points = 0;
    HIPCHK(hipMalloc(&h->d_large2, cg_large_bytes(n)));
    HIPCHK(hipMemset(h->d_large2, 0, cg_large_bytes(n)));
    cg_large_layout(h->d_large2, n, h->lg2);
    if (!h->h_meta2) HIPCHK(hipHostMalloc((void**)&h->h_meta2, LG_META_WORDS * 4, hipHostMallocDefault));
    h->lg2.hmeta = h->h_meta2;
    h->large2_points = n;
    return CG_OK;
}

// Work enqueued on stream s reuses the handle's result and scratch slots: when the handle's last
// work went to another stream, s waits for it (the handle's calls stay ordered whatever stream
// each names). Calls on one stream pay nothing.
int order_after_last(cg_handle* h, hipStream_t s) {
    if (!h->last_stream || h->last_stream == s) return CG_OK;
    if (!h->ev_switch) HIPCHK(hipEventCreateWithFlags(&h->ev_switch, hipEventDisableTiming));
    HIPCHK(hipEventRecord(h->ev_switch, h->last_stream));
    HIPCHK(hipStreamWaitEvent(s, h->ev_switch, 0));
    return CG_OK;
}

// order_after_last, then s is the handle's last stream (entry points that enqueue on the
// handle's buffers)
int use_stream(cg_handle* h, hipStream_t s) {
    int rc = order_after_last(h, s);
    if (!rc) h->last_stream = s;
    return rc;
}

// The next launch's span slot (cg_debug_launch_spans), or null.
unsigned long long* take_span(cg_handle* h) {
    if (!h->spans_left) return nullptr;
    unsigned long long* p = h->next_span;
    h->next_span += CG_SPAN_WORDS;
    h->spans_left--;
    return p;
}

int launch_frames(cg_handle* h, CgLaunch& L, int kmode, hipStream_t s) {
    const bool large = L.n_points > CG_MAX_POINTS || ((h->route == 1 || h->route == 2 || h->route == 5) && L.n_points > 0);
    if (!large && L.split) {
        HIPCHK((hipError_t)cg_launch_split(L, h->dp, kmode, s));
        return CG_OK;
    }
    if (!large) {   // one fused workgroup per frame
        HIPCHK((hipError_t)cg_launch_batch(L, h->dp, kmode, s));
        return CG_OK;
    }
    int rc = ensure_large(h, L.n_points);
    if (rc) return rc;
    L.stamps = nullptr;
    const bool dev_sized = kmode != CG_KMODE_GROUND && h->dp.voxel_order == CG_VOXEL_ORDER_PCL &&
                           L.n_points <= LG_DEV_MAX_POINTS;
    if (L.n_frames > 1 && kmode != CG_KMODE_GROUND && !dev_sized) {   // two scratch sets: frames pipelined
        rc = ensure_large2(h, L.n_points);
        if (rc) return rc;
        const LgScratch S2 = route_scratch(h, true);
        HIPCHK((hipError_t)cg_run_large(L, h->dp, kmode, route_scratch(h), s, &S2));
        return CG_OK;
    }
    // (the hint is whatever the last finished frame wrote: no synchronisation)
    uint32_t hint[LG_HINT_WORDS] = {};
    for (int k = 0; h->h_hint && k < LG_HINT_WORDS; k++) hint[k] = __atomic_load_n(h->h_hint + k, __ATOMIC_RELAXED);
    HIPCHK((hipError_t)cg_run_large(L, h->dp, kmode, route_scratch(h), s, nullptr, &h->lg_graphs,
                                    h->h_hint ? hint : nullptr));
    return CG_OK;
}

int ensure_pack(cg_handle* h) {
    if (!h->d_pack) {
        HIPCHK(hipMalloc(&h->d_pack, CG_PACK_WORDS * 4));
        // coherent: the split kernel's done word follows its packed words there (CG_PACK_DONE)
        HIPCHK(hipHostMalloc((void**)&h->h_pack, CG_PACK_WORDS * 4, hipHostMallocCoherent));
        std::memset(h->h_pack, 0, CG_PACK_WORDS * 4);
        HIPCHK(hipHostGetDevicePointer((void**)&h->h_pack_dev, h->h_pack, 0));
    }
    return CG_OK;
}

#ifndef CG_PACK_SPIN_US
#define CG_PACK_SPIN_US 2000
#endif
// true once *w == seq (acquire: the packed words before it are visible), false after
// CG_PACK_SPIN_US microseconds
bool wait_done_word(const uint32_t* w, uint32_t seq) {
    if (!CG_HOOK_POLL_DONE_WORD) return false;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t k = 1;; k++) {
        if (__atomic_load_n(w, __ATOMIC_ACQUIRE) == seq) return true;
        __builtin_ia32_pause();
        if ((k & 255) == 0 &&
            std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(CG_PACK_SPIN_US))
            return false;
    }
}

int fetch_frame(cg_handle* h, hipStream_t s, uint32_t frame, cg_detect_result* out) {
    const uint64_t cap = h->cap_points;
    // one packed copy into pinned memory and one synchronisation when the results fit
    // CG_PACK_MAX entries per array (every frame of the LDS backend: V <= M <= CG_MMAX); the
    // single-frame split launch packs into the pinned buffer itself (no copy)
    int rc = ensure_pack(h);
    if (rc) return rc;
    {
        CgLaunch L{};   // the result arrays only (fill_launch_outputs would reset the stamps)
        L.cap = h->cap_points;
        L.hdr = h->d_hdr; L.vox = h->d_vox; L.lab = h->d_lab; L.offs = h->d_offs;
        L.idx = h->d_idx; L.cen = h->d_cen;
        const bool prepacked = h->packed && frame == 0;   // by the single-frame launch just run
        const uint32_t done = prepacked ? h->pack_seq : 0u;
        h->packed = false;
        if (!prepacked) {
            HIPCHK((hipError_t)cg_launch_pack(L, frame, h->d_pack, s));
            // every word but the done word: d_pack's copy of it is never written, and a stale
            // value there must not land where the next split call's wait polls
            HIPCHK(hipMemcpyAsync(h->h_pack, h->d_pack, CG_PACK_DONE * 4, hipMemcpyDeviceToHost, s));
        }
        // the split launch's done word, polled in host memory (no runtime call); a frame still
        // running after CG_PACK_SPIN_US (a slow backend, a staging timeout) waits on the stream
        if (!(done && wait_done_word(h->h_pack + CG_PACK_DONE, done))) HIPCHK(cg_stream_wait(s));
        const uint32_t* p = h->h_pack;
        const uint32_t V = p[CG_HDR_V], C = p[CG_HDR_C];
        if (V <= CG_PACK_MAX && C <= CG_PACK_MAX && (C == 0 || p[CG_PACK_OFFS + C] <= CG_PACK_MAX)) {
            std::memcpy(h->h_hdr, p, CG_HDR_WORDS * 4);
            if (p[CG_HDR_ERR] == CG_HDR_E_WAIT)
                return fail(CG_E_DEVICE, "frame %u: a device-side wait of the large-frame path gave up; results void", frame);
            out->n_points = p[CG_HDR_N];
            out->n_kept = p[CG_HDR_K];
            out->n_filtered = p[CG_HDR_M];
            out->n_voxels = V;
            out->n_clusters = C;
            out->flags = p[CG_HDR_FLAGS];
            out->voxels = (float*)(h->h_pack + CG_PACK_VOX);
            out->labels = (int32_t*)(h->h_pack + CG_PACK_LAB);
            out->cluster_offsets = (int32_t*)(h->h_pack + CG_PACK_OFFS);
            out->cluster_indices = (int32_t*)(h->h_pack + CG_PACK_IDX);
            out->centroids = (float*)(h->h_pack + CG_PACK_CEN);
            return CG_OK;
        }
    }
    HIPCHK(hipMemcpyAsync(h->h_hdr, h->d_hdr + (uint64_t)frame * CG_HDR_WORDS, CG_HDR_WORDS * 4,
                          hipMemcpyDeviceToHost, s));
    HIPCHK(cg_stream_wait(s));
    if (h->h_hdr[CG_HDR_ERR] == CG_HDR_E_WAIT)
        return fail(CG_E_DEVICE, "frame %u: a device-side wait of the large-frame path gave up; results void", frame);
    const uint32_t V = h->h_hdr[CG_HDR_V], C = h->h_hdr[CG_HDR_C];
    h->h_vox.resize((size_t)V * 4 + 4);
    h->h_lab.resize((size_t)V + 1);
    h->h_offs.resize((size_t)C + 2);
    h->h_cen.resize((size_t)C * 2 + 2);
    h->h_idx.resize((size_t)V + 1);
    if (V) {
        HIPCHK(hipMemcpyAsync(h->h_vox.data(), h->d_vox + frame * cap, (size_t)V * 16, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(h->h_lab.data(), h->d_lab + frame * cap, (size_t)V * 4, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipMemcpyAsync(h->h_offs.data(), h->d_offs + frame * (cap + 1), (size_t)(C + 1) * 4,
                          hipMemcpyDeviceToHost, s));
    if (C) {
        HIPCHK(hipMemcpyAsync(h->h_cen.data(), h->d_cen + frame * cap, (size_t)C * 8, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(cg_stream_wait(s));
    const uint32_t nidx = C ? (uint32_t)h->h_offs[C] : 0u;
    if (nidx) {
        HIPCHK(hipMemcpyAsync(h->h_idx.data(), h->d_idx + frame * cap, (size_t)nidx * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(cg_stream_wait(s));
    }
    out->n_points = h->h_hdr[CG_HDR_N];
    out->n_kept = h->h_hdr[CG_HDR_K];
    out->n_filtered = h->h_hdr[CG_HDR_M];
    out->n_voxels = V;
    out->n_clusters = C;
    out->flags = h->h_hdr[CG_HDR_FLAGS];
    out->voxels = h->h_vox.data();
    out->labels = h->h_lab.data();
    out->cluster_offsets = h->h_offs.data();
    out->cluster_indices = h->h_idx.data();
    out->centroids = h->h_cen.data();
    return CG_OK;
}

// The staging buffer's chunks (CG_SPLIT_CHUNK points each): copied from the message (unless
// `only_flags`: already staged) and published to the split kernel's chunk workgroups one by
// one (release: the chunk's bytes before its word).
StagePool* stage_pool(cg_handle* h) {
    if (h->pool || h->pool_tried) return h->pool;
    h->pool_tried = true;
    const char* e = std::getenv("CG_STAGE_THREADS");
    const int k = e ? std::atoi(e) : 3;
    if (k <= 0) return nullptr;
    StagePool* p = new StagePool();
    p->parts = (uint32_t)std::min(k, 15) + 1u;
    if (const char* sp = std::getenv("CG_STAGE_SPIN_US")) p->spin_ns = (uint64_t)std::atoll(sp) * 1000ull;
    try {
        for (uint32_t t = 1; t < p->parts; t++) p->th.emplace_back([p, t] { p->worker(t); });
    } catch (...) {   // (no threads: the caller copies alone)
        delete p;
        return nullptr;
    }
    h->pool = p;
    return p;
}

void publish_chunks(cg_handle* h, const cg_cloud_view* v, uint32_t n, uint32_t step, bool only_flags) {
    // every workgroup of the launch waits for its word: one even for an empty frame
    const uint32_t nch = std::max<uint32_t>(1, (n + CG_SPLIT_CHUNK - 1) / CG_SPLIT_CHUNK);
    const uint8_t* src = (const uint8_t*)v->data;
    StagePool* pool = nch > 1 ? stage_pool(h) : nullptr;
    if (pool) {   // interleaved chunks: helpers take parts 1.., the caller part 0
        pool->src = src; pool->dst = h->h_stage; pool->flags = h->h_flags;
        pool->seq = h->stage_seq; pool->n = n; pool->step = step; pool->nch = nch; pool->copy = !only_flags;
        pool->left.store(pool->parts - 1, std::memory_order_relaxed);
        pool->job.store(pool->job.load(std::memory_order_relaxed) + 1u, std::memory_order_release);
        if (pool->sleepers.load() > 0) {
            std::lock_guard<std::mutex> lk(pool->mu);
            pool->cv.notify_all();
        }
        pool->chunks(0);
        // the message is the caller's until the call returns: the helpers finish with it first
        while (pool->left.load(std::memory_order_acquire)) _mm_pause();
        return;
    }
    for (uint32_t c = 0; c < nch; c++) {
        if (!only_flags && (uint64_t)c * CG_SPLIT_CHUNK < n) {
            const size_t b0 = (size_t)c * CG_SPLIT_CHUNK * step;
            const size_t nb = (size_t)std::min<uint32_t>(CG_SPLIT_CHUNK, n - c * CG_SPLIT_CHUNK) * step;
            std::memcpy(h->h_stage + b0, src + b0, nb);
        }
        __atomic_thread_fence(__ATOMIC_SEQ_CST);   // also orders a memcpy's non-temporal stores
        __atomic_store_n(&h->h_flags[c], h->stage_seq, __ATOMIC_RELEASE);
    }
}

// Retries (the call is then only slower, never failed):
//   RETRY_DMA: the frame again with its input staged whole and copied by DMA (route 4's form),
//   after a zero-copy call whose chunk workgroups gave up waiting for the host's publish words
//   (a host thread descheduled for CG_STAGE_TIMEOUT);
//   RETRY_ONE_WG: the frame again in one workgroup (route 3's form), after a split launch whose
//   chunk workgroups gave up waiting for each other (CG_SPLIT_TIMEOUT: other work held the CUs).
enum { RETRY_DMA = 1, RETRY_ONE_WG = 2 };
int run_single(cg_handle* h, const cg_cloud_view* in, int kmode, cg_detect_result* dres,
               cg_ground_result* gres, int retry = 0) {
    const bool dma_retry = (retry & RETRY_DMA) != 0;
    if (!h) return fail(CG_E_INVALID, "null handle");
    int rc = check_view(in);
    if (rc) return rc;
    HIPCHK(hipSetDevice(h->device));
    rc = own_stream(h);
    if (rc) return rc;
    if ((rc = order_after_last(h, h->stream))) return rc;
    const uint32_t n = in->width * in->height;
    rc = ensure_batch(h, 1, n, kmode == CG_KMODE_GROUND);
    if (rc) return rc;
    CgLaunch L{};
    // a frame alone on the GPU: pass 1 over one workgroup per 4,096-point chunk (route 3:
    // the one-workgroup frame kernel, for comparisons)
    const bool split = kmode != CG_KMODE_GROUND && n <= CG_MAX_POINTS &&
                       (h->route == 0 || h->route == 4 || h->route == 6 || h->route == 9) && !(retry & RETRY_ONE_WG);
    bool staged_later = false;
    // route 4: split, input by DMA; route 6 (tests): zero-copy with no chunk ever published
    // route 9 (tests): zero-copy with chunk workgroup 0 giving up on the others at once
    const bool zero_copy = split && (h->route == 0 || h->route == 6 || h->route == 9) && !dma_retry;
    rc = stage_frame(h, in, L, zero_copy, &staged_later);
    if (rc) return rc;
    fill_launch_outputs(h, L);
    h->last_single = false;
    if (kmode == CG_KMODE_PIPELINE) {
        L.seckeys = h->d_seckeys;
    }
    if (zero_copy) {   // the input's chunks published after the launch
        if (!h->h_flags) {
            HIPCHK(hipHostMalloc((void**)&h->h_flags, 64 * 4, hipHostMallocCoherent));
            std::memset(h->h_flags, 0, 64 * 4);
            HIPCHK(hipHostGetDevicePointer((void**)&h->h_flags_dev, h->h_flags, 0));
        }
        h->stage_seq = h->stage_seq + 1 ? h->stage_seq + 1 : 1;
        L.in_flags = h->h_flags_dev;
        L.in_seq = h->stage_seq;
        if (!staged_later && h->route != 6) publish_chunks(h, in, n, 0, true);   // already staged: publish every chunk
    }
    if (split) {
        if (!h->d_split) {
            HIPCHK(hipMalloc(&h->d_split, CG_SPLIT_WORDS * 4));
            // the state words as the kernel's last workgroup leaves them: zero, the minima all ones
            HIPCHK(hipMemsetAsync(h->d_split, 0, SP_STATE * 4, h->stream));
            HIPCHK(hipMemsetAsync(h->d_split + SP_KEYS, 0xff, (CG_NUM_BINS + 1) * 4, h->stream));
            HIPCHK(hipMemsetAsync(h->d_split + SP_BMIN, 0xff, 3 * 4, h->stream));
        }
        L.split = h->d_split;
        rc = ensure_pack(h);
        if (rc) return rc;
        L.pack = h->h_pack_dev;   // the kernel packs the results itself, into pinned host memory
        h->pack_seq = h->pack_seq + 1 ? h->pack_seq + 1 : 1;
        L.pack_seq = h->pack_seq;
        L.split_give_up = h->route == 9 ? 1u : 0u;
    }
    h->packed = L.pack != nullptr;
    rc = launch_frames(h, L, kmode, h->stream);
    if (rc) return rc;
    if (staged_later && h->route != 6) publish_chunks(h, in, n, L.point_step, false);   // overlaps the chunk workgroups
    h->last_frames = 1; h->last_points = n; h->last_mode = kmode; h->last_stream = h->stream;
    h->last_in = L;
    if (kmode == CG_KMODE_GROUND) {
        const size_t bytes = std::max<size_t>((size_t)n * 32, 32);
        if (bytes > h->h_ground_bytes) {
            if (h->h_ground) (void)hipHostFree(h->h_ground);
            h->h_ground = nullptr;
            HIPCHK(hipHostMalloc(&h->h_ground, bytes, hipHostMallocDefault));
            h->h_ground_bytes = bytes;
        }
        if (n) HIPCHK(hipMemcpyAsync(h->h_ground, h->d_ground, (size_t)n * 32, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(hipMemcpyAsync(h->h_hdr, h->d_hdr, CG_HDR_WORDS * 4, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(cg_stream_wait(h->stream));
        gres->n_points = n;
        gres->n_kept = h->h_hdr[CG_HDR_K];
        gres->width = in->width;
        gres->height = in->height;
        gres->data = h->h_ground;
        return CG_OK;
    }
    rc = fetch_frame(h, h->stream, 0, dres);
    if (rc) return rc;
    if (L.in_flags && __atomic_load_n(&h->h_flags[CG_STAGE_ERR], __ATOMIC_ACQUIRE) == L.in_seq) {
        // a chunk was processed before its bytes were published: the results are void; the
        // staging buffer is complete now, so the frame runs again with its input by DMA
        h->retries++;
        return run_single(h, in, kmode, dres, gres, retry | RETRY_DMA);
    }
    if (split && h->h_hdr[CG_HDR_ERR]) {   // (the kernel's own flag: header word 7)
        h->retries++;
        return run_single(h, in, kmode, dres, gres, retry | RETRY_ONE_WG);
    }
    h->last_k = h->h_hdr[CG_HDR_K];
    h->last_single = true;
    return CG_OK;
}

// get_reconstructed_cone's box (src/cone_detection.cpp:228-229) as exact float bounds:
// (double)x <= (double)cx + (double)0.228f / 1.5  <=>  x <= floor_to_float(that double sum)
RcBox crop_box(float cx, float cy) {
    const double w = (double)0.228f / 1.5;   // CONE_WIDTH is a const float (line 22)
    RcBox b;
    b.lox = cg_ceil_to_float((double)cx - w);
    b.hix = cg_floor_to_float((double)cx + w);
    b.loy = cg_ceil_to_float((double)cy - w);
    b.hiy = cg_floor_to_float((double)cy + w);
    return b;
}

}  // namespace

extern "C" {

// 0.2.0: cg_run_batch_split, cg_debug_front_span and CG_F_PAIR_TIMEOUT removed (round 4;
// INTEGRATION.md, ABI history)
const char* cg_version(void) { return "cones_gpu 0.2.1 (gfx950)"; }

void cg_params_init(cg_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->num_of_sectors = 16;                 // src/ground_removal.cpp:18
    p->default_lowest_point = -0.1f;        // src/ground_removal.cpp:19
    p->distance_treshold_max = 7.0;         // src/cone_detection.cpp:27
    p->distance_treshold_min = 0.7;         // :28
    p->level_threshold = -0.5;              // :29
    p->angle_threshold = 90.0;              // :30
    p->min_cluster_size = 3;                // :32
    p->max_cluster_size = 50;               // :33
    p->cones_matching_dist_theshold = 0.5;  // :39
    p->cone_position_extension_length = 0.05;  // :40
    p->voxel_filter_leaf_size_x = 0.04;     // :41-43
    p->voxel_filter_leaf_size_y = 0.04;
    p->voxel_filter_leaf_size_z = 0.04;
}

int cg_create(const cg_params* params, int device, cg_handle** out) {
    if (!out) return fail(CG_E_INVALID, "null output handle pointer");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(CG_E_DEVICE, "no HIP device");
    if (device < 0 || device >= ndev) return fail(CG_E_DEVICE, "device %d out of range (%d)", device, ndev);
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(CG_E_DEVICE, "device %d is %s; this library is built for gfx950", device, prop.gcnArchName);
    cg_params p;
    if (params) p = *params; else cg_params_init(&p);
    CgDevParams dp;
    int rc = prepare(p, dp);
    if (rc) return rc;
    dp.voxel_order = CG_VOXEL_ORDER_PCL;
    HIPCHK(hipSetDevice(device));
    cg_handle* h = new cg_handle();
    h->device = device;
    h->params = p;
    h->dp = dp;
    *out = h;   // the handle's own stream is created on first use (see own_stream)
    return CG_OK;
}

int cg_destroy(cg_handle* h) {
    if (!h) return CG_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)cg_stream_wait(h->stream);
    free_batch(h);
    if (h->ev_switch) (void)hipEventDestroy(h->ev_switch);
    if (h->d_stamps) (void)hipFree(h->d_stamps);
    if (h->d_in) (void)hipFree(h->d_in);
    if (h->h_meta) (void)hipHostFree(h->h_meta);
    if (h->h_hint) (void)hipHostFree(h->h_hint);
    if (h->d_large) (void)hipFree(h->d_large);
    cg_large_graphs_free(h->lg_graphs);
    if (h->h_meta2) (void)hipHostFree(h->h_meta2);
    if (h->d_large2) (void)hipFree(h->d_large2);
    if (h->d_cn_w) (void)hipFree(h->d_cn_w);
    if (h->d_cn_pts) (void)hipFree(h->d_cn_pts);
    if (h->d_cn_offs) (void)hipFree(h->d_cn_offs);
    if (h->d_pack) (void)hipFree(h->d_pack);
    if (h->h_pack) (void)hipHostFree(h->h_pack);
    if (h->d_split) (void)hipFree(h->d_split);
    if (h->d_boxes) (void)hipFree(h->d_boxes);
    if (h->d_rc_cnt) (void)hipFree(h->d_rc_cnt);
    if (h->d_rc_out) (void)hipFree(h->d_rc_out);
    delete h->pool;   // (joins the helpers; none is copying: every call waits for its helpers)
    if (h->h_stage) (void)hipHostFree(h->h_stage);
    if (h->h_flags) (void)hipHostFree(h->h_flags);
    if (h->h_ground) (void)hipHostFree(h->h_ground);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return CG_OK;
}

int cg_set_params(cg_handle* h, const cg_params* params) {
    if (!h || !params) return fail(CG_E_INVALID, "null argument");
    CgDevParams dp;
    int rc = prepare(*params, dp);
    if (rc) return rc;
    dp.voxel_order = h->dp.voxel_order;
    h->params = *params;
    h->dp = dp;
    return CG_OK;
}

int cg_set_voxel_order(cg_handle* h, int order) {
    if (!h) return fail(CG_E_INVALID, "null handle");
    if (order != CG_VOXEL_ORDER_POINT && order != CG_VOXEL_ORDER_PCL)
        return fail(CG_E_INVALID, "unknown voxel order %d", order);
    h->dp.voxel_order = order;
    return CG_OK;
}

int cg_ground_remove(cg_handle* h, const cg_cloud_view* in, cg_ground_result* out) {
    if (!out) return fail(CG_E_INVALID, "null result");
    return run_single(h, in, CG_KMODE_GROUND, nullptr, out);
}
int cg_detect(cg_handle* h, const cg_cloud_view* in, cg_detect_result* out) {
    if (!out) return fail(CG_E_INVALID, "null result");
    return run_single(h, in, CG_KMODE_DETECT, out, nullptr);
}
int cg_pipeline(cg_handle* h, const cg_cloud_view* in, cg_detect_result* out) {
    if (!out) return fail(CG_E_INVALID, "null result");
    return run_single(h, in, CG_KMODE_PIPELINE, out, nullptr);
}

// The re-crop of one frame L (frame 0 of L) whose detector input was the groundless cloud
// (pipe: sector keys at d_seckeys, K kept points) or the frame itself.
static int recrop_frame(cg_handle* h, const CgLaunch& L, bool pipe, const uint32_t* d_seckeys, uint32_t K,
                        const float* centers_xy, uint32_t n_centers, cg_crop_result* out) {
    const uint32_t N = L.n_points, nblk = cg_recrop_blocks(N);
    const uint32_t npad = pipe ? N - K : 0u;   // the groundless cloud's PointXYZI() tail
    h->h_rc_off.assign((size_t)n_centers + 1, 0u);
    h->h_rc_pts.clear();
    std::vector<RcBox> boxes(std::min<uint32_t>(n_centers, CG_RECROP_MAX_BOXES));
    if (!h->d_boxes && n_centers) HIPCHK(hipMalloc(&h->d_boxes, CG_RECROP_MAX_BOXES * sizeof(RcBox)));
    for (uint32_t c0 = 0; c0 < n_centers; c0 += CG_RECROP_MAX_BOXES) {
        const uint32_t nb = std::min<uint32_t>(CG_RECROP_MAX_BOXES, n_centers - c0);
        for (uint32_t b = 0; b < nb; b++) boxes[b] = crop_box(centers_xy[2 * (c0 + b)], centers_xy[2 * (c0 + b) + 1]);
        const size_t ncnt = (size_t)nb * nblk;
        if (2 * ncnt > h->rc_cnt_cap) {
            (void)hipFree(h->d_rc_cnt);
            h->d_rc_cnt = nullptr;
            h->rc_cnt_cap = 0;
            HIPCHK(hipMalloc(&h->d_rc_cnt, 2 * ncnt * 4));
            h->rc_cnt_cap = 2 * ncnt;
        }
        HIPCHK(hipMemcpyAsync(h->d_boxes, boxes.data(), nb * sizeof(RcBox), hipMemcpyHostToDevice, h->stream));
        h->h_rc_cnt.assign(ncnt, 0u);
        if (ncnt) {
            HIPCHK((hipError_t)cg_launch_recrop(L, h->dp, pipe, d_seckeys, h->d_boxes, nb, h->d_rc_cnt, nullptr,
                                                nullptr, false, h->stream));
            HIPCHK(hipMemcpyAsync(h->h_rc_cnt.data(), h->d_rc_cnt, ncnt * 4, hipMemcpyDeviceToHost, h->stream));
            HIPCHK(cg_stream_wait(h->stream));
        }
        // device slots: box-major, blocks in order
        std::vector<uint32_t> off(ncnt), box_lo(nb), box_n(nb, 0u);
        uint64_t total = 0;
        for (size_t q = 0; q < ncnt; q++) {
            if (q % nblk == 0) box_lo[q / nblk] = (uint32_t)total;
            off[q] = (uint32_t)total;
            total += h->h_rc_cnt[q];
            box_n[q / nblk] += h->h_rc_cnt[q];
        }
        if (total > 0xffffffffull) return fail(CG_E_CAPACITY, "re-crop output exceeds 2^32 points");
        h->h_rc_dev.assign((size_t)total * 4, 0.f);
        if (total) {
            if (total > h->rc_out_cap) {
                (void)hipFree(h->d_rc_out);
                h->d_rc_out = nullptr;
                h->rc_out_cap = 0;
                HIPCHK(hipMalloc(&h->d_rc_out, total * 16));
                h->rc_out_cap = total;
            }
            HIPCHK(hipMemcpyAsync(h->d_rc_cnt + ncnt, off.data(), ncnt * 4, hipMemcpyHostToDevice, h->stream));
            HIPCHK((hipError_t)cg_launch_recrop(L, h->dp, pipe, d_seckeys, h->d_boxes, nb, nullptr,
                                                h->d_rc_cnt + ncnt, h->d_rc_out, true, h->stream));
            HIPCHK(hipMemcpyAsync(h->h_rc_dev.data(), h->d_rc_out, total * 16, hipMemcpyDeviceToHost, h->stream));
            HIPCHK(cg_stream_wait(h->stream));
        }
        // each box: its device points in cloud order, then the zero pads if the box holds the origin
        for (uint32_t b = 0; b < nb; b++) {
            const size_t lo = box_lo[b], hi = lo + box_n[b];
            h->h_rc_pts.insert(h->h_rc_pts.end(), h->h_rc_dev.begin() + 4 * lo, h->h_rc_dev.begin() + 4 * hi);
            const RcBox& x = boxes[b];
            if (npad && 0.f >= x.lox && 0.f <= x.hix && 0.f >= x.loy && 0.f <= x.hiy)
                h->h_rc_pts.insert(h->h_rc_pts.end(), (size_t)npad * 4, 0.f);
            h->h_rc_off[c0 + b + 1] = (uint32_t)(h->h_rc_pts.size() / 4);
        }
    }
    out->n_centers = n_centers;
    out->offsets = h->h_rc_off.data();
    out->points = h->h_rc_pts.empty() ? nullptr : h->h_rc_pts.data();
    return CG_OK;
}

int cg_recrop(cg_handle* h, const float* centers_xy, uint32_t n_centers, cg_crop_result* out) {
    if (!h || !out || (n_centers && !centers_xy)) return fail(CG_E_INVALID, "null argument");
    if (!h->last_single || (h->last_mode != CG_KMODE_DETECT && h->last_mode != CG_KMODE_PIPELINE))
        return fail(CG_E_INVALID, "cg_recrop needs a preceding cg_detect or cg_pipeline call on the handle");
    HIPCHK(hipSetDevice(h->device));
    int rc = own_stream(h);
    if (rc) return rc;
    return recrop_frame(h, h->last_in, h->last_mode == CG_KMODE_PIPELINE, h->d_seckeys, h->last_k, centers_xy,
                        n_centers, out);
}

int cg_batch_recrop(cg_handle* h, uint32_t frame, const float* centers_xy, uint32_t n_centers, cg_crop_result* out) {
    if (!h || !out || (n_centers && !centers_xy)) return fail(CG_E_INVALID, "null argument");
    if (!h->batch_valid) return fail(CG_E_INVALID, "cg_batch_recrop needs a preceding cg_run_batch on the handle");
    if (frame >= h->last_batch.n_frames)
        return fail(CG_E_INVALID, "frame %u >= %u", frame, h->last_batch.n_frames);
    HIPCHK(hipSetDevice(h->device));
    int rc = own_stream(h);
    if (rc) return rc;
    // the batch ran on its own stream: its header (K) after it finishes
    uint32_t hdr[CG_HDR_WORDS];
    HIPCHK(hipMemcpyAsync(hdr, h->d_hdr + (uint64_t)frame * CG_HDR_WORDS, sizeof(hdr), hipMemcpyDeviceToHost,
                          h->last_stream));
    HIPCHK(cg_stream_wait(h->last_stream));
    CgLaunch L = h->last_batch;
    L.in += (uint64_t)frame * L.frame_stride;
    L.n_frames = 1;
    const bool pipe = h->batch_kmode == CG_KMODE_PIPELINE;
    return recrop_frame(h, L, pipe, h->d_seckeys + (uint64_t)frame * (CG_NUM_BINS + 1), hdr[CG_HDR_K], centers_xy,
                        n_centers, out);
}

namespace {
int check_batch(const cg_batch* b, int mode) {
    if (!b) return fail(CG_E_INVALID, "null batch");
    if (mode != CG_MODE_PIPELINE && mode != CG_MODE_DETECT) return fail(CG_E_INVALID, "bad mode %d", mode);
    if (b->n_points > CG_MAX_FRAME_POINTS)
        return fail(CG_E_CAPACITY, "frames of %u points; the engine supports <= %u", b->n_points,
                    (unsigned)CG_MAX_FRAME_POINTS);
    if (b->n_frames && b->n_points && !b->d_data) return fail(CG_E_INVALID, "null batch data");
    if (b->point_step == 0 || b->point_step % 4 || b->frame_stride % 4 ||
        b->frame_stride < (uint64_t)b->n_points * b->point_step)
        return fail(CG_E_INVALID, "bad point_step / frame_stride");
    const int32_t offs[4] = {b->off_x, b->off_y, b->off_z, b->off_intensity};
    for (int32_t o : offs)
        if (o >= 0 && (o % 4 || (uint32_t)o + 4 > b->point_step))
            return fail(CG_E_INVALID, "field offset %d invalid for point_step %u", o, b->point_step);
    return CG_OK;
}

// One checked batch call on the handle's device (already current).
int run_batch(cg_handle* h, const cg_batch* b, int mode, void* hip_stream) {
    int rc = ensure_batch(h, b->n_frames, b->n_points, false);
    if (rc) return rc;
    CgLaunch L{};
    L.in = (const uint8_t*)b->d_data;
    L.frame_stride = b->frame_stride;
    L.n_frames = b->n_frames;
    L.n_points = b->n_points;
    L.point_step = b->point_step;
    L.off_x = b->off_x; L.off_y = b->off_y; L.off_z = b->off_z; L.off_i = b->off_intensity;
    L.is_dense = b->is_dense;
    fill_launch_outputs(h, L);
    if (!hip_stream) {
        rc = own_stream(h);
        if (rc) return rc;
    }
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : h->stream;
    if ((rc = order_after_last(h, s))) return rc;
    L.span = take_span(h);
    const int kmode = mode == CG_MODE_PIPELINE ? CG_KMODE_PIPELINE : CG_KMODE_DETECT;
    if (kmode == CG_KMODE_PIPELINE) L.seckeys = h->d_seckeys;   // per frame, for cg_batch_recrop
    rc = launch_frames(h, L, kmode, s);
    if (rc) return rc;
    h->last_batch = L;
    h->batch_kmode = kmode;
    h->batch_valid = true;
    h->last_frames = b->n_frames; h->last_points = b->n_points; h->last_mode = mode;
    h->last_stream = s;
    h->last_single = false;
    return CG_OK;
}
}  // namespace

int cg_run_batch(cg_handle* h, const cg_batch* b, int mode, void* hip_stream) {
    if (!h || !b) return fail(CG_E_INVALID, "null argument");
    int rc = check_batch(b, mode);
    if (rc) return rc;
    HIPCHK(hipSetDevice(h->device));
    return run_batch(h, b, mode, hip_stream);
}

int cg_run_batches(cg_handle* const* handles, const cg_batch* batches, uint32_t n_calls, int mode,
                   void* const* hip_streams, uint32_t* n_done) {
    if (n_done) *n_done = 0;
    if (n_calls && (!handles || !batches || !hip_streams)) return fail(CG_E_INVALID, "null argument");
    for (uint32_t i = 0; i < n_calls; i++) {   // every call checked before any is enqueued
        if (!handles[i]) return fail(CG_E_INVALID, "null handle at call %u", i);
        int rc = check_batch(&batches[i], mode);
        if (rc) return rc;
    }
    int dev = -1;
    for (uint32_t i = 0; i < n_calls; i++) {
        cg_handle* h = handles[i];
        if (h->device != dev) {
            HIPCHK(hipSetDevice(h->device));
            dev = h->device;
        }
        int rc = run_batch(h, &batches[i], mode, hip_streams[i]);
        if (rc) return rc;
        if (n_done) *n_done = i + 1;
    }
    return CG_OK;
}

int cg_batch_results_get(cg_handle* h, cg_batch_results* out) {
    if (!h || !out) return fail(CG_E_INVALID, "null argument");
    out->n_frames = h->last_frames;
    out->capacity = h->cap_points;
    out->d_header = h->d_hdr;
    out->d_voxels = (const float*)h->d_vox;
    out->d_labels = h->d_lab;
    out->d_cluster_offsets = h->d_offs;
    out->d_cluster_indices = h->d_idx;
    out->d_centroids = (const float*)h->d_cen;
    return CG_OK;
}

int cg_batch_fetch(cg_handle* h, uint32_t frame, cg_detect_result* out) {
    if (!h || !out) return fail(CG_E_INVALID, "null argument");
    if (frame >= h->last_frames) return fail(CG_E_INVALID, "frame %u >= %u", frame, h->last_frames);
    HIPCHK(hipSetDevice(h->device));
    const int rc = fetch_frame(h, h->last_stream, frame, out);
    if (rc == CG_OK && h->h_hdr[CG_HDR_ERR] != 0u)   // (include/cones_gpu.h CG_HDR_ERR)
        return fail(CG_E_DEVICE, "frame %u: header error word %#x; results void", frame, h->h_hdr[CG_HDR_ERR]);
    return rc;
}

// ---- tiled frames (C5) ----------------------------------------------------------------------
namespace {
CgLaunch tile_launch(const cg_tile& t) {
    CgLaunch L{};
    L.in = (const uint8_t*)t.d_data;
    L.n_frames = 1;
    L.n_points = t.n;
    L.frame_stride = (uint64_t)t.n * t.point_step;
    L.point_step = t.point_step;
    L.off_x = t.off_x; L.off_y = t.off_y; L.off_z = t.off_z; L.off_i = t.off_intensity;
    L.is_dense = 0;
    return L;
}
}  // namespace

int cg_tile_front(cg_handle* h, const cg_tile* t, uint32_t* keys) {
    if (!h || !t || !keys) return fail(CG_E_INVALID, "null argument");
    if (t->n && !t->d_data) return fail(CG_E_INVALID, "null tile data");
    if (t->n_total > CG_MAX_FRAME_POINTS || (uint64_t)t->first + t->n > t->n_total)
        return fail(CG_E_INVALID, "tile [%u, %u + %u) outside a frame of %u points", t->first, t->first, t->n, t->n_total);
    if (t->point_step == 0 || t->point_step % 4) return fail(CG_E_INVALID, "bad point_step");
    const int32_t offs[4] = {t->off_x, t->off_y, t->off_z, t->off_intensity};
    for (int32_t o : offs)
        if (o >= 0 && (o % 4 || (uint32_t)o + 4 > t->point_step)) return fail(CG_E_INVALID, "bad field offset %d", o);
    HIPCHK(hipSetDevice(h->device));
    int rc = own_stream(h);
    if (rc) return rc;
    rc = ensure_large(h, std::max<uint32_t>(t->n, 1));
    if (!rc) rc = use_stream(h, h->stream);
    if (rc) return rc;
    h->tile = *t;
    CgLaunch L = tile_launch(*t);
    LgScratch S = route_scratch(h);
    S.pidx_base = t->first;
    HIPCHK((hipError_t)cg_large_front(L, h->dp, CG_KMODE_PIPELINE, S, h->stream, 0, true));
    HIPCHK(hipMemcpyAsync(keys, S.meta + LG_SECKEY, CG_TILE_KEYS * 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(cg_stream_wait(h->stream));
    h->tile_ready = true;
    return CG_OK;
}

int cg_tile_decide(cg_handle* h, const uint32_t* merged_keys, uint32_t* counts) {
    if (!h || !merged_keys || !counts) return fail(CG_E_INVALID, "null argument");
    if (!h->tile_ready) return fail(CG_E_INVALID, "cg_tile_decide before cg_tile_front");
    HIPCHK(hipSetDevice(h->device));
    if (int rc = use_stream(h, h->stream)) return rc;
    LgScratch S = route_scratch(h);
    S.pidx_base = h->tile.first;
    HIPCHK(hipMemcpyAsync(S.meta + LG_SECKEY, merged_keys, CG_TILE_KEYS * 4, hipMemcpyHostToDevice, h->stream));
    CgLaunch L = tile_launch(h->tile);
    HIPCHK((hipError_t)cg_large_decide(L, h->dp, S, h->stream, 0));
    uint32_t m[LG_META_WORDS];
    HIPCHK(hipMemcpyAsync(m, S.meta, sizeof(m), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(cg_stream_wait(h->stream));
    counts[0] = m[LG_K];
    counts[1] = m[LG_MS];
    counts[2] = m[LG_NFIN];
    for (int a = 0; a < 3; a++) { counts[3 + a] = m[LG_BMIN + a]; counts[6 + a] = m[LG_BMAX + a]; }
    return CG_OK;
}

int cg_tile_survivors(cg_handle* h, float* d_points, uint32_t* d_index, uint32_t capacity) {
    if (!h) return fail(CG_E_INVALID, "null handle");
    if (!h->tile_ready) return fail(CG_E_INVALID, "cg_tile_survivors before cg_tile_front");
    HIPCHK(hipSetDevice(h->device));
    if (int rc = use_stream(h, h->stream)) return rc;
    uint32_t n = 0;
    HIPCHK(hipMemcpyAsync(&n, h->lg.meta + LG_MS, 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(cg_stream_wait(h->stream));
    if (n > capacity) return fail(CG_E_INVALID, "%u survivors do not fit %u", n, capacity);
    if (n && (!d_points || !d_index)) return fail(CG_E_INVALID, "null output buffers");
    if (n) {
        HIPCHK(hipMemcpyAsync(d_points, h->lg.surv_p, (size_t)n * 16, hipMemcpyDeviceToDevice, h->stream));
        HIPCHK(hipMemcpyAsync(d_index, h->lg.surv_i, (size_t)n * 4, hipMemcpyDeviceToDevice, h->stream));
    }
    HIPCHK(cg_stream_wait(h->stream));
    return CG_OK;
}

int cg_tile_backend(cg_handle* h, const float* d_points, const uint32_t* d_index, uint32_t n_survivors,
                    const uint32_t* merged_counts, uint32_t n_total) {
    if (!h || !merged_counts) return fail(CG_E_INVALID, "null argument");
    if (n_survivors && (!d_points || !d_index)) return fail(CG_E_INVALID, "null survivors");
    if (n_total == 0 || n_total > CG_MAX_FRAME_POINTS || n_survivors > n_total || merged_counts[0] > n_total ||
        merged_counts[1] != n_survivors)
        return fail(CG_E_INVALID, "inconsistent tile counts (%u survivors, K %u, N %u)", n_survivors,
                    merged_counts[0], n_total);
    HIPCHK(hipSetDevice(h->device));
    int rc = own_stream(h);
    if (rc) return rc;
    rc = ensure_large(h, n_total);
    if (rc) return rc;
    rc = ensure_batch(h, 1, n_total, false);
    if (!rc) rc = use_stream(h, h->stream);
    if (rc) return rc;
    LgScratch S = route_scratch(h);
    S.pidx_base = 0;
    HIPCHK((hipError_t)cg_large_set_survivors(S, h->dp, d_points, d_index, n_survivors, merged_counts, h->stream));
    CgLaunch L{};
    L.n_frames = 1;
    L.n_points = n_total;
    fill_launch_outputs(h, L);
    L.stamps = nullptr;
    HIPCHK((hipError_t)cg_large_backend(L, h->dp, CG_KMODE_PIPELINE, S, h->stream, 0, n_total, merged_counts[0]));
    HIPCHK(cg_stream_wait(h->stream));
    h->last_frames = 1; h->last_points = n_total; h->last_mode = CG_MODE_PIPELINE; h->last_stream = h->stream;
    h->last_single = false;
    return CG_OK;
}

// ---- the tile protocol with device-side keys and counts (no synchronisation) ----------------
namespace {
int tile_check(const cg_tile* t) { return cg_check_tile(t); }
}  // namespace

int cg_tile_front_async(cg_handle* h, const cg_tile* t, uint32_t* d_keys, void* hip_stream) {
    if (!h || !t || !d_keys) return fail(CG_E_INVALID, "null argument");
    int rc = tile_check(t);
    if (rc) return rc;
    HIPCHK(hipSetDevice(h->device));
    if ((rc = own_stream(h))) return rc;
    if ((rc = ensure_large(h, std::max<uint32_t>(t->n, 1)))) return rc;
    const hipStream_t s = hip_stream ? (hipStream_t)hip_stream : h->stream;
    if ((rc = use_stream(h, s))) return rc;
    h->tile = *t;
    LgScratch S = route_scratch(h);
    S.pidx_base = t->first;
    HIPCHK((hipError_t)cg_large_front(tile_launch(*t), h->dp, CG_KMODE_PIPELINE, S, s, 0, true));
    HIPCHK(hipMemcpyAsync(d_keys, S.meta + LG_SECKEY, CG_TILE_KEYS * 4, hipMemcpyDeviceToDevice, s));
    h->tile_ready = true;
    return CG_OK;
}

int cg_tile_decide_async(cg_handle* h, const uint32_t* d_merged_keys, uint32_t* d_counts, void* hip_stream) {
    if (!h || !d_merged_keys || !d_counts) return fail(CG_E_INVALID, "null argument");
    if (!h->tile_ready) return fail(CG_E_INVALID, "cg_tile_decide_async before cg_tile_front_async");
    HIPCHK(hipSetDevice(h->device));
    const hipStream_t s = hip_stream ? (hipStream_t)hip_stream : h->stream;
    if (int rc = use_stream(h, s)) return rc;
    LgScratch S = route_scratch(h);
    S.pidx_base = h->tile.first;
    HIPCHK(hipMemcpyAsync(S.meta + LG_SECKEY, d_merged_keys, CG_TILE_KEYS * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK((hipError_t)cg_large_decide(tile_launch(h->tile), h->dp, S, s, 0));
    HIPCHK((hipError_t)cg_large_tile_counts(S, d_counts, s));
    return CG_OK;
}

int cg_tile_survivors_async(cg_handle* h, float* d_points, uint32_t* d_index, uint32_t n, void* hip_stream) {
    if (!h) return fail(CG_E_INVALID, "null handle");
    if (!h->tile_ready) return fail(CG_E_INVALID, "cg_tile_survivors_async before cg_tile_front_async");
    if (n > std::max<uint32_t>(h->tile.n, 1)) return fail(CG_E_INVALID, "%u survivors in a tile of %u points", n, h->tile.n);
    if (n && (!d_points || !d_index)) return fail(CG_E_INVALID, "null output buffers");
    HIPCHK(hipSetDevice(h->device));
    const hipStream_t s = hip_stream ? (hipStream_t)hip_stream : h->stream;
    if (int rc = use_stream(h, s)) return rc;
    if (n) {
        HIPCHK(hipMemcpyAsync(d_points, h->lg.surv_p, (size_t)n * 16, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(d_index, h->lg.surv_i, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
    }
    return CG_OK;
}

int cg_tile_backend_own(cg_handle* h, uint32_t n_total, void* hip_stream) {
    if (!h) return fail(CG_E_INVALID, "null handle");
    if (!h->tile_ready) return fail(CG_E_INVALID, "cg_tile_backend_own before cg_tile_decide_async");
    if (h->tile.first != 0 || h->tile.n != n_total || h->tile.n_total != n_total)
        return fail(CG_E_INVALID, "cg_tile_backend_own needs the whole frame in the tile ([%u, %u + %u) of %u)",
                    h->tile.first, h->tile.first, h->tile.n, n_total);
    HIPCHK(hipSetDevice(h->device));
    int rc = ensure_batch(h, 1, n_total, false);
    if (rc) return rc;
    const hipStream_t s = hip_stream ? (hipStream_t)hip_stream : h->stream;
    if ((rc = use_stream(h, s))) return rc;
    LgScratch S = route_scratch(h);
    S.pidx_base = 0;
    CgLaunch L{};
    L.n_frames = 1;
    L.n_points = n_total;
    fill_launch_outputs(h, L);
    L.stamps = nullptr;
    // the survivors and the counts (the whole frame's) are where cg_tile_decide_async left them
    HIPCHK((hipError_t)cg_large_backend(L, h->dp, CG_KMODE_PIPELINE, S, s, 0, n_total, CG_K_FROM_META));
    h->last_frames = 1; h->last_points = n_total; h->last_mode = CG_MODE_PIPELINE; h->last_stream = s;
    h->last_single = false;
    h->batch_valid = false;
    return CG_OK;
}

// ---- C5 halo tiling (cg_halo_*): argument checks and the handle's scratch; the work is in
// cg_large.hip
namespace {
int halo_counts_ok(const uint32_t* c, uint32_t n_total) { return cg_halo_counts_check(c, n_total); }
int halo_plan_ok(const cg_halo_plan* p) { return cg_halo_plan_check(p); }
}  // namespace

int cg_halo_plan_frame(cg_handle* h, const uint32_t* merged_counts, uint32_t n_total, uint32_t n_ranks,
                       cg_halo_plan* plan) {
    if (!h || !plan) return fail(CG_E_INVALID, "null argument");
    int rc = halo_counts_ok(merged_counts, n_total);
    if (rc) return rc;
    cg_halo_plan_compute(h->dp, merged_counts, n_total, n_ranks, plan);
    return CG_OK;
}

int cg_halo_owner(cg_handle* h, const cg_halo_plan* plan, const float* d_points, uint32_t n, int32_t* d_slab) {
    if (!h) return fail(CG_E_INVALID, "null handle");
    int rc = halo_plan_ok(plan);
    if (rc) return rc;
    if (n && (!d_points || !d_slab)) return fail(CG_E_INVALID, "null buffers");
    HIPCHK(hipSetDevice(h->device));
    rc = own_stream(h);
    if (!rc) rc = use_stream(h, h->stream);
    if (rc) return rc;
    HIPCHK((hipError_t)cg_launch_halo_owner(d_points, n, h->dp.inv_leaf[0], plan->min_b[0], plan->slab_w, plan->slabs,
                                            d_slab, h->stream));
    HIPCHK(cg_stream_wait(h->stream));
    return CG_OK;
}

int cg_halo_local(cg_handle* h, const cg_halo_plan* plan, const float* d_points, const uint32_t* d_index,
                  uint32_t n, uint32_t n_pads, const uint32_t* merged_counts, uint32_t n_total, uint32_t* d_rec,
                  uint32_t capacity, uint32_t* n_vox) {
    if (!h || !n_vox) return fail(CG_E_INVALID, "null argument");
    int rc = halo_plan_ok(plan);
    if (!rc) rc = halo_counts_ok(merged_counts, n_total);
    if (rc) return rc;
    if (n && (!d_points || !d_index)) return fail(CG_E_INVALID, "null survivors");
    if (plan->slabs == 1) {
        // one slab has no boundary: its backend is the frame's, run on every survivor (non-finite
        // ones included, as cg_tile_backend) in frame-index voxel order, results in the handle
        if (n != merged_counts[1] || n_pads != plan->n_pads)
            return fail(CG_E_INVALID, "one slab takes all %u survivors and %u pads (got %u + %u)", merged_counts[1],
                        plan->n_pads, n, n_pads);
        HIPCHK(hipSetDevice(h->device));
        rc = own_stream(h);
        if (!rc) rc = ensure_large(h, n_total);
        if (!rc) rc = ensure_batch(h, 1, n_total, false);
        if (!rc) rc = use_stream(h, h->stream);
        if (rc) return rc;
        LgScratch S = route_scratch(h);
        S.pidx_base = 0;
        HIPCHK((hipError_t)cg_large_set_survivors(S, h->dp, d_points, d_index, n, merged_counts, h->stream));
        CgLaunch L{};
        L.n_frames = 1;
        L.n_points = n_total;
        fill_launch_outputs(h, L);
        L.stamps = nullptr;
        CgDevParams Pm = h->dp;
        Pm.voxel_order = CG_VOXEL_ORDER_POINT;
        HIPCHK((hipError_t)cg_large_backend(L, Pm, CG_KMODE_PIPELINE, S, h->stream, 0, n_total, merged_counts[0]));
        h->last_frames = 1; h->last_points = n_total; h->last_mode = CG_MODE_PIPELINE; h->last_stream = h->stream;
        h->last_single = false;
        h->batch_valid = false;
        *n_vox = 0;
        return CG_OK;
    }
    if ((uint64_t)n + n_pads > n_total || n > merged_counts[2] || (n_pads && n_pads != plan->n_pads))
        return fail(CG_E_INVALID, "%u survivors + %u pads do not fit the frame's counts", n, n_pads);
    if ((uint64_t)n + n_pads > capacity || (capacity && !d_rec))
        return fail(CG_E_INVALID, "record capacity %u < %u possible voxels", capacity, n + n_pads);
    HIPCHK(hipSetDevice(h->device));
    rc = own_stream(h);
    if (!rc) rc = ensure_large(h, n_total);
    if (!rc) rc = ensure_batch(h, 1, n_total, false);
    if (!rc) rc = use_stream(h, h->stream);
    if (rc) return rc;
    LgScratch S = route_scratch(h);
    S.pidx_base = 0;
    CgLaunch L{};
    L.n_frames = 1;
    L.n_points = n_total;
    fill_launch_outputs(h, L);
    L.stamps = nullptr;
    HIPCHK((hipError_t)cg_halo_local_run(L, h->dp, S, h->stream, d_points, d_index, n, n_pads, plan->n_pads,
                                         merged_counts, n_total, plan->key_bits, d_rec, capacity, n_vox));
    return CG_OK;
}

int cg_halo_edges(cg_handle* h, const uint32_t* d_own, uint32_t n_own, const uint32_t* d_halo, uint32_t n_halo,
                  uint32_t* d_pairs, uint32_t capacity, uint32_t* n_pairs) {
    if (!h || !n_pairs) return fail(CG_E_INVALID, "null argument");
    if ((n_own && !d_own) || (n_halo && !d_halo) || (capacity && !d_pairs)) return fail(CG_E_INVALID, "null buffers");
    HIPCHK(hipSetDevice(h->device));
    int rc = own_stream(h);
    if (!rc) rc = ensure_large(h, 1);
    if (!rc) rc = use_stream(h, h->stream);
    if (rc) return rc;
    uint32_t* d_count = h->lg.meta + LG_META_WORDS - 1;
    HIPCHK((hipError_t)cg_halo_edges_run(d_own, n_own, d_halo, n_halo, h->dp.r2, d_pairs, capacity, d_count,
                                         h->stream));
    HIPCHK(hipMemcpyAsync(n_pairs, d_count, 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(cg_stream_wait(h->stream));
    return CG_OK;
}

int cg_halo_merge(cg_handle* h, const cg_halo_plan* plan, const uint32_t* d_rec, uint32_t n_rec,
                  const uint32_t* d_pairs, uint32_t n_pairs, const uint32_t* merged_counts, uint32_t n_total) {
    if (!h) return fail(CG_E_INVALID, "null handle");
    int rc = halo_plan_ok(plan);
    if (!rc) rc = halo_counts_ok(merged_counts, n_total);
    if (rc) return rc;
    if ((n_rec && !d_rec) || (n_pairs && !d_pairs)) return fail(CG_E_INVALID, "null buffers");
    const uint64_t Mtot = (uint64_t)merged_counts[1] + plan->n_pads;
    if (n_rec > Mtot) return fail(CG_E_INVALID, "%u voxel records for %llu detector points", n_rec,
                                  (unsigned long long)Mtot);
    HIPCHK(hipSetDevice(h->device));
    rc = own_stream(h);
    if (!rc) rc = ensure_large(h, n_total);
    if (!rc) rc = ensure_batch(h, 1, n_total, false);
    if (!rc) rc = use_stream(h, h->stream);
    if (rc) return rc;
    LgScratch S = route_scratch(h);
    S.pidx_base = 0;
    CgLaunch L{};
    L.n_frames = 1;
    L.n_points = n_total;
    fill_launch_outputs(h, L);
    L.stamps = nullptr;
    HIPCHK((hipError_t)cg_halo_merge_run(L, h->dp, S, h->stream, d_rec, n_rec, d_pairs, n_pairs, plan->key_bits,
                                         (uint32_t)Mtot, merged_counts[0]));
    HIPCHK(cg_stream_wait(h->stream));
    h->last_frames = 1; h->last_points = n_total; h->last_mode = CG_MODE_PIPELINE; h->last_stream = h->stream;
    h->last_single = false;
    return CG_OK;
}

// ---- colour classifier (cg_colornet.hip) --------------------------------------------------
int cg_colornet_set(cg_handle* h, const float* weights, uint32_t n_weights) {
    if (!h || !weights) return fail(CG_E_INVALID, "null argument");
    if (n_weights != CG_COLORNET_WEIGHTS)
        return fail(CG_E_INVALID, "colour net weights: %u floats, expected %u", n_weights, CG_COLORNET_WEIGHTS);
    HIPCHK(hipSetDevice(h->device));
    int rc = own_stream(h);
    if (rc) return rc;
    if (!h->d_cn_w) HIPCHK(hipMalloc(&h->d_cn_w, CG_COLORNET_WEIGHTS * sizeof(float)));
    HIPCHK(hipMemcpyAsync(h->d_cn_w, weights, CG_COLORNET_WEIGHTS * sizeof(float), hipMemcpyHostToDevice, h->stream));
    HIPCHK(cg_stream_wait(h->stream));
    return CG_OK;
}

int cg_classify_colors(cg_handle* h, const float* points, const uint32_t* offsets, uint32_t n_cones,
                       int32_t* colors, float* probs, uint8_t* images) {
    if (!h || !offsets || (n_cones && !colors)) return fail(CG_E_INVALID, "null argument");
    if (!h->d_cn_w) return fail(CG_E_INVALID, "no colour net weights: call cg_colornet_set first");
    if (n_cones == 0) return CG_OK;
    if (offsets[0] != 0) return fail(CG_E_INVALID, "offsets[0] must be 0");
    for (uint32_t c = 0; c < n_cones; c++)
        if (offsets[c + 1] < offsets[c]) return fail(CG_E_INVALID, "offsets decrease at cone %u", c);
    const uint32_t np = offsets[n_cones];
    if (np && !points) return fail(CG_E_INVALID, "null points");
    HIPCHK(hipSetDevice(h->device));
    int rc = own_stream(h);
    if (rc) return rc;
    if (np > h->cn_pts_cap) {
        if (h->d_cn_pts) HIPCHK(hipFree(h->d_cn_pts));
        h->d_cn_pts = nullptr;
        h->cn_pts_cap = std::max<size_t>(np, 4096);
        HIPCHK(hipMalloc(&h->d_cn_pts, h->cn_pts_cap * sizeof(float4)));
    }
    // per cone: offset (n + 1), colour, 3 probabilities, 180 image bytes (45 words)
    const size_t words = (size_t)n_cones + 1 + n_cones + 3 * (size_t)n_cones + 45 * (size_t)n_cones;
    if (words > h->cn_cap) {
        if (h->d_cn_offs) HIPCHK(hipFree(h->d_cn_offs));
        h->d_cn_offs = nullptr;
        h->cn_cap = std::max<size_t>(words, 1024);
        HIPCHK(hipMalloc(&h->d_cn_offs, h->cn_cap * 4));
    }
    uint32_t* d_offs = h->d_cn_offs;
    int32_t* d_col = (int32_t*)(d_offs + n_cones + 1);
    float* d_prob = (float*)(d_col + n_cones);
    uint8_t* d_img = (uint8_t*)(d_prob + 3 * (size_t)n_cones);
    if (np) HIPCHK(hipMemcpyAsync(h->d_cn_pts, points, (size_t)np * 16, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(d_offs, offsets, ((size_t)n_cones + 1) * 4, hipMemcpyHostToDevice, h->stream));
    HIPCHK((hipError_t)cg_launch_colornet(h->d_cn_pts, d_offs, n_cones, h->d_cn_w, d_col, d_prob,
                                          images ? d_img : nullptr, h->stream));
    HIPCHK(hipMemcpyAsync(colors, d_col, (size_t)n_cones * 4, hipMemcpyDeviceToHost, h->stream));
    if (probs) HIPCHK(hipMemcpyAsync(probs, d_prob, (size_t)n_cones * 12, hipMemcpyDeviceToHost, h->stream));
    if (images) HIPCHK(hipMemcpyAsync(images, d_img, (size_t)n_cones * 180, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(cg_stream_wait(h->stream));
    return CG_OK;
}

int cg_debug_large_meta(cg_handle* h, uint32_t* out, uint32_t n_words) {
    return cg_debug_large_buffer(h, 0, out, (uint64_t)n_words * 4);
}

int cg_debug_large_buffer(cg_handle* h, int which, void* out, uint64_t bytes) {
    if (!h || !out) return fail(CG_E_INVALID, "null argument");
    if (!h->d_large) return fail(CG_E_INVALID, "no large frame has run on this handle");
    // 4: the first 1024 bytes of the radix histogram area (phase stamps of variant builds,
    // tools/variants/lg_stamps.h)
    const void* src = which == 0   ? (const void*)h->lg.meta
                      : which == 1 ? (const void*)h->lg.codes
                      : which == 2 ? (const void*)h->lg.keep
                      : which == 4 ? (const void*)h->lg.hist
                                   : (const void*)h->lg.pq;
    const uint64_t nch = ((uint64_t)h->large_points + LG_CHUNK - 1) / LG_CHUNK;
    const uint64_t cap = which == 0   ? LG_META_WORDS * 4
                         : which == 1 ? nch * LG_CHUNK
                         : which == 2 ? nch * CG_BLOCK * 16
                         : which == 4 ? CG_DEBUG_HIST_BYTES
                                      : (uint64_t)cg_large_pq_words() * 4;
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(out, src, std::min(bytes, cap), hipMemcpyDeviceToHost));
    return CG_OK;
}

int cg_debug_launch_span(cg_handle* h, void* d_span) { return cg_debug_launch_spans(h, d_span, d_span ? 1u : 0u); }

int cg_debug_launch_spans(cg_handle* h, void* d_spans, uint32_t n_launches) {
    if (!h) return fail(CG_E_INVALID, "null handle");
    if (n_launches && !d_spans) return fail(CG_E_INVALID, "null span buffer");
    h->next_span = (unsigned long long*)d_spans;
    h->spans_left = n_launches;
    return CG_OK;
}

int cg_debug_route(cg_handle* h, int route) {
    if (!h) return fail(CG_E_INVALID, "null handle");
    if (route < 0 || (route > 6 && route != 9 && route != 10)) return fail(CG_E_INVALID, "bad route %d", route);   // (7, 8: retired experiments)
    h->route = route;
    return CG_OK;
}

int cg_debug_stamps(cg_handle* h, int enable) {
    if (!h) return fail(CG_E_INVALID, "null handle");
    HIPCHK(hipSetDevice(h->device));
    h->stamps_on = enable != 0;
    if (!h->stamps_on && h->d_stamps) {
        (void)hipFree(h->d_stamps);
        h->d_stamps = nullptr;
        h->stamps_frames = 0;
    }
    return CG_OK;
}

int cg_debug_stamps_fetch(cg_handle* h, uint64_t* out, uint32_t n_frames) {
    if (!h || !out) return fail(CG_E_INVALID, "null argument");
    if (!h->d_stamps || n_frames > h->stamps_frames) return fail(CG_E_INVALID, "stamps not enabled");
    HIPCHK(hipSetDevice(h->device));
    if (h->last_stream) HIPCHK(cg_stream_wait(h->last_stream));
    HIPCHK(hipMemcpy(out, h->d_stamps, (size_t)n_frames * 32 * 8, hipMemcpyDeviceToHost));
    return CG_OK;
}

int cg_selftest_atan2f(cg_handle* h, const float* y, const float* x, float* out, uint32_t n) {
    if (!h || (n && (!y || !x || !out))) return fail(CG_E_INVALID, "null argument");
    if (!n) return CG_OK;
    HIPCHK(hipSetDevice(h->device));
    int rc = own_stream(h);
    if (rc) return rc;
    float *dy = nullptr, *dx = nullptr, *dout = nullptr;
    HIPCHK(hipMalloc(&dy, (size_t)n * 4));
    HIPCHK(hipMalloc(&dx, (size_t)n * 4));
    HIPCHK(hipMalloc(&dout, (size_t)n * 8));
    HIPCHK(hipMemcpy(dy, y, (size_t)n * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dx, x, (size_t)n * 4, hipMemcpyHostToDevice));
    HIPCHK((hipError_t)cg_launch_selftest_atan2f(dy, dx, dout, n, h->stream));
    HIPCHK(cg_stream_wait(h->stream));
    HIPCHK(hipMemcpy(out, dout, (size_t)n * 8, hipMemcpyDeviceToHost));
    (void)hipFree(dy); (void)hipFree(dx); (void)hipFree(dout);
    return CG_OK;
}

int cg_selftest_sqrt(cg_handle* h, const double* s, double* out, uint32_t n) {
    if (!h || (n && (!s || !out))) return fail(CG_E_INVALID, "null argument");
    if (!n) return CG_OK;
    HIPCHK(hipSetDevice(h->device));
    int rc = own_stream(h);
    if (rc) return rc;
    double *din = nullptr, *dout = nullptr;
    HIPCHK(hipMalloc(&din, (size_t)n * 8));
    HIPCHK(hipMalloc(&dout, (size_t)n * 8));
    HIPCHK(hipMemcpy(din, s, (size_t)n * 8, hipMemcpyHostToDevice));
    HIPCHK((hipError_t)cg_launch_selftest_sqrt(din, dout, n, h->stream));
    HIPCHK(cg_stream_wait(h->stream));
    HIPCHK(hipMemcpy(out, dout, (size_t)n * 8, hipMemcpyDeviceToHost));
    (void)hipFree(din); (void)hipFree(dout);
    return CG_OK;
}

}  // extern "C"
