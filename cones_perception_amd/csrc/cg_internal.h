// cg_internal.h — structures shared by the HIP kernels (cg_kernels.hip) and the host side of
// the C-ABI (cg_api.cpp). Not part of the public boundary (include/cones_gpu.h).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

// Device form of cg_params: the reference's float-vs-double comparisons pre-resolved on the
// host into exact float / double thresholds (see cg_math.h and DESIGN.md §Numerics).
struct CgDevParams {
    float  default_low;     // default_lowest_point (src/ground_removal.cpp:19,58)
    float  level_f;         // remove iff z < level_f    <=> (double)z < level_threshold
    double s_far;           // remove iff S >= s_far      <=> euclidan_dist > distance_treshold_max
    double s_near;          // remove iff S <  s_near     <=> euclidan_dist < distance_treshold_min
    float  ang_lo;          // remove iff a <= ang_lo     <=> -theta >= atan2f(y,x)
    float  ang_hi;          // remove iff a >= ang_hi     <=> atan2f(y,x) >= theta
    float  inv_leaf[3];     // VoxelGrid inverse_leaf_size_ = 1.0f / (float)leaf
    float  r2;              // float(tol * tol), tol = float(sqrt(0.325f^2 + 0.228f^2))
    float  cell_inv;        // 1 / neighbour-grid cell size (cell = 1.0625 * tol)
    uint32_t min_cl, max_cl;// cluster size limits as PCL's unsigned compares see them
    double ext;             // cone_position_extension_length
    int32_t zero_pass;      // a (0,0,0,i=0) pad point survives filter_points_position
    // fast-path certificates (float bounds around the exact double thresholds): a float
    // sum of squares below *_lo / above *_hi decides the compare without the double path
    float sfar_lo, sfar_hi, snear_lo, snear_hi;
    // 8-bit z code window for the on-chip ground decision (cg_device.h zcode):
    // d(z) = sat_u8(rne(fl(zq_bias - 64 z))), d(zq_z0) = 1 for the highest possible threshold
    float zq_z0, zq_bias;
    // angle-filter certificates: |a| >= ang_cert_hi removes and |a| < ang_cert_lo keeps for
    // every exact angle within CG_ANG_MARGIN of the fast approximation a
    float ang_cert_lo, ang_cert_hi;
    // sector rays for the coherent fast path (cg_device.h ray_inside): sector s is the wedge
    // between the unit vectors ray[s].xy = (cos, sin)(s * SEC) and ray[s].zw at its upper
    // edge ((s + 1) * SEC; 2 pi for sector 16). ray_filter_ok: sectors whose whole wedge (plus
    // CG_RAY_WEDGE_PAD) lies on one side of the angle filter; ray_arm: those it removes.
    float4 ray[17];
    uint32_t ray_filter_ok, ray_arm;
    // voxel summation order (cg_set_voxel_order): CG_VOXEL_ORDER_PCL = PCL's std::sort
    // permutation (cg_pcl.h), CG_VOXEL_ORDER_POINT = ascending point index
    int32_t voxel_order;
};

// Sets the thread-local message cg_last_error returns; returns code.
int cg_set_error(int code, const char* msg);

// Certified fast angle classification (cg_device.h classify_angle_fast): the approximation's
// error bound is 2.3e-6 rad (polynomial, v_rcp_f32 and roundings 2.0e-6 against the true
// atan2, glibc's own rounding 2.4e-7); decisions are certified only farther than these
// margins from a boundary (radians / sector units), everything else takes the exact path.
#define CG_ANG_MARGIN 8.0e-6f
#define CG_SEC_MARGIN_T 2.5e-5f
// Sector-ray certificate: a point is certified inside its lane's current sector when both
// edge cross products clear CG_RAY_EPS * (|x| + |y|), i.e. its true angle lies >= 1.9e-5 rad
// inside the wedge, against <= 8.5e-7 rad between the true edge and the reference's own
// floor(fl(wrap(atan2f)) / SEC) edge. The angle-filter class of a sector is decided over the
// wedge widened by CG_RAY_WEDGE_PAD on both sides.
#define CG_RAY_EPS 2.0e-5f
#define CG_RAY_WEDGE_PAD 1.0e-4

// One batch launch: uniform frames, device-resident input and outputs.
struct CgLaunch {
    const uint8_t* in;
    uint64_t frame_stride;
    uint32_t n_frames, n_points, point_step;
    int32_t off_x, off_y, off_z, off_i;
    uint32_t is_dense;
    // outputs (per frame slots of `cap` points)
    uint32_t cap;
    uint32_t* hdr;      // n_frames x 8
    float4*  vox;       // n_frames x cap
    int32_t* lab;       // n_frames x cap
    int32_t* offs;      // n_frames x (cap + 1)
    int32_t* idx;       // n_frames x cap
    float2*  cen;       // n_frames x cap
    uint8_t* ground;    // n_frames x n_points x 32 B (ground-only mode)
    // HBM scratch for frames whose survivors do not fit the LDS path
    uint8_t* scratch;
    uint64_t scratch_stride;
    // diagnostics: per-workgroup phase timestamps (16 slots per frame) or null
    uint64_t* stamps;
    // per-frame final sector-minimum keys (18 words) for cg_recrop, or null (ground modes)
    uint32_t* seckeys;
    // timing: [first workgroup start, last workgroup end] of the launch (s_memrealtime,
    // 100 MHz), or null (cg_debug_launch_span)
    unsigned long long* span;
    // split single-frame launch (cg_launch_split): CG_SPLIT_WORDS of state, or null
    uint32_t* split;
    // split launch: the frame's results also packed here (CG_PACK_WORDS) at the end, or null
    uint32_t* pack;
    // split launch: the frame in pinned host memory; each chunk workgroup copies its chunk to
    // `in` (the device copy) before pass 1, or null (`in` already holds the frame)
    const uint8_t* in_host;
    // split launch with in_host: the host fills the staging buffer chunk by chunk after the
    // launch and publishes chunk c by storing in_seq to in_flags[c] (pinned, coherent); each
    // chunk workgroup waits for its word (CG_STAGE_TIMEOUT bound: then in_flags[CG_STAGE_ERR]
    // is set and the call fails). Null: the buffer is complete before the launch.
    uint32_t* in_flags;
    uint32_t in_seq;
    // split launch with pack: the last workgroup stores pack_seq to pack[CG_PACK_DONE] once
    // every packed word is in host memory (the host returns on it; 0: no done word)
    uint32_t pack_seq;
    // split launch, tests (cg_debug_route 9): chunk workgroup 0 gives up at once instead of
    // waiting for the others, as after a CG_SPLIT_TIMEOUT
    uint32_t split_give_up;
};
#define CG_STAGE_ERR 63               // in_flags word set by a chunk workgroup that timed out
#define CG_STAGE_TIMEOUT 20000000ull  // s_memrealtime ticks (100 MHz): 200 ms
// A single frame of <= CG_MAX_POINTS points spread over one workgroup per 4,096-point chunk:
// pass 1 per chunk; once every chunk's sector minima are merged, pass 2 and the survivors per
// chunk; the last chunk to finish gathers the survivors and runs the backend. State words (SP_*,
// reset by the last workgroup; the host zeroes them once, keys and bounds minima to all ones),
// then the frame's survivors: x, y, z, intensity (float4) and point index per slot.
#define CG_SPLIT_CHUNK (8 * CG_BLOCK)   // 8 points per lane: one uint2 of codes, one byte of bits
enum {
    SP_ARRIVE = 0,      // chunks whose sector minima are merged
    SP_TOUCHED = 1,     // used sector bins (OR)
    SP_KEYS = 2,        // 18 sector-minimum keys (MIN)
    SP_DONE = 20,       // chunks done with their survivors
    SP_MS, SP_K,        // survivors, kept points (SUM)
    SP_BMIN, SP_BMAX = SP_BMIN + 3, SP_NFIN = SP_BMAX + 3,   // VoxelGrid bounds keys, finite survivors
    SP_ERR,             // a chunk gave up waiting for the others (CG_SPLIT_TIMEOUT)
    SP_STATE = 64,
    SP_SURV = SP_STATE
};
#define CG_SPLIT_WORDS (SP_SURV + 5 * CG_MAX_POINTS)
#define CG_SPLIT_TIMEOUT 40000000ull   // s_memrealtime ticks (100 MHz): 400 ms
int cg_launch_split(const CgLaunch& L, const CgDevParams& P, int kmode, hipStream_t s);

// Hooks for experiment builds. tools/build_variant.sh force-includes a header from
// tools/variants/ that may define them (a kernel stopping after a phase, a spinning stream wait,
// the done-word poll off); the product build leaves them as below.
//   CG_HOOK_FRAME_PHASE(k): the frame kernel after phase k (1 pass 1, 2 pass 2 and the
//     survivor gather, 3 the pads and bounds), every thread, with L, f, N and tid in scope
//   CG_HOOK_STREAM_WAIT(s): the host's wait for a stream's queued work
//   CG_HOOK_POLL_DONE_WORD: 0 makes fetch_frame wait on the stream instead of the done word
#ifndef CG_HOOK_FRAME_PHASE
#define CG_HOOK_FRAME_PHASE(k) ((void)0)
#endif
#ifndef CG_HOOK_STREAM_WAIT
#define CG_HOOK_STREAM_WAIT(s) hipStreamSynchronize(s)
#endif
#ifndef CG_HOOK_POLL_DONE_WORD
#define CG_HOOK_POLL_DONE_WORD 1
#endif
//   CG_HOOK_LG_STAMP(S, i): a large-frame kernel's phase i (lg_cluster_tail), thread 0 of the
//     workgroup, with the LgScratch S in scope
#ifndef CG_HOOK_LG_STAMP
#define CG_HOOK_LG_STAMP(S, i) ((void)0)
#endif
//   CG_HOOK_PQF(S, t, k, v): lg_pq_flow's ticket t, record word k (0 entry taken, 1 split done,
//     2 range word complete, 3 end, 4 first | last << 32, 5 entry word | first ticket << 32),
//     thread 0, with the LgScratch S in scope (tools/variants/pqf_stamps.h)
#ifndef CG_HOOK_PQF
#define CG_HOOK_PQF(S, t, k, v) ((void)0)
#endif
#ifndef CG_DEBUG_HIST_BYTES
#define CG_DEBUG_HIST_BYTES 1024   // cg_debug_large_buffer(4): bytes of the histogram area returned
#endif

// Host wait for a stream's queued work.
static inline hipError_t cg_stream_wait(hipStream_t s) { return CG_HOOK_STREAM_WAIT(s); }

#ifndef CG_BLOCK
#define CG_BLOCK 512           // one workgroup (8 waves) per frame, two per CU
#endif
#ifndef CG_MMAX
#define CG_MMAX 1024           // LDS-path capacity (points surviving the filter)
#endif
#define CG_MAX_POINTS 65536    // frame kernel: 128 points per lane; larger frames: cg_large.hip
#define CG_MAX_FRAME_POINTS (1u << 28)

enum { CG_LAYOUT_GENERIC = 0, CG_LAYOUT_XYZI16 = 1, CG_LAYOUT_PCL32 = 2 };
enum { CG_KMODE_PIPELINE = 0, CG_KMODE_DETECT = 1, CG_KMODE_GROUND = 2 };

// ---- frames of more than CG_MAX_POINTS points (cg_large.hip) ----
// dense neighbour grid of the global backend: at most LG_DGRID_AXIS cells per axis
#define LG_DGRID_AXIS 128
#define LG_DCELLS_MAX (LG_DGRID_AXIS * LG_DGRID_AXIS * LG_DGRID_AXIS)
// per-chunk statistics words (LgScratch::cstat)
enum { LG_CS_KEYS = 0, LG_CS_TOUCHED = 18, LG_CS_K, LG_CS_MS, LG_CS_BMIN, LG_CS_BMAX = LG_CS_BMIN + 3,
       LG_CS_NFIN = LG_CS_BMAX + 3, LG_CS_WORDS = 32 };
#define LG_CHUNK 4096          // points per front workgroup (8 per lane): a 1M frame fills 256
// per-frame meta words in HBM
enum {
    LG_SECKEY = 0,             // 18 words: sector minima (order-preserving keys)
    LG_TOUCHED = 18, LG_K, LG_UNSORTED, LG_MS, LG_NFIN,
    LG_BMIN, LG_BMAX = LG_BMIN + 3, LG_V = LG_BMAX + 3, LG_C, LG_U, LG_PASS,
    LG_MINB, LG_MUL1 = LG_MINB + 3, LG_MUL2, LG_ORG, LG_NFIN_ALL = LG_ORG + 3, LG_SCAN_N,
    LG_DGINV, LG_DGN = LG_DGINV + 3, LG_NCELL = LG_DGN + 3,   // dense neighbour grid
    LG_SORT_LIM,               // cluster-order sort: key bits in use (digits past it are skipped)
    LG_PCL_N,                  // PCL voxel order: finite points in index_vector (compaction total)
    // the backend sized on the device (cg_run_large): written by the decisions' fold
    LG_MALL,                   //   detector input points M = survivors + pads
    LG_MTOT,                   //   M for the global backend's launches (0 when the LDS backend runs)
    LG_NPAD,                   //   PointXYZI() pads after the kept points
    LG_KHDR,                   //   K for the header
    LG_SMALL,                  //   1: the LDS backend (one workgroup) takes the frame
    LG_PQ_TIMEOUT,             // a partition level's wait for its range gave up (never expected)
    LG_META_WORDS = 64
};
struct LgScratch {
    uint32_t* meta;
    uint64_t* codes;          // z codes, [chunk][group][lane] words of 8
    uint64_t* keep;           // per chunk and lane: kept bits (ground-only mode), else filter bits
                              // (pipeline, until lg_decide leaves the survivor bits there)
    uint32_t* chunk_cnt;      // ground-only mode: kept points per chunk
    float4* surv_p; uint32_t* surv_i;   // survivors (detector input points)
    uint64_t* key0; uint64_t* key1;     // radix sort ping-pong
    uint32_t* val0; uint32_t* val1;
    uint32_t* hist;           // 256 x tiles + 1
    uint32_t* sstat;          // single-pass scan status words (tickets, finished, per tile)
    float4* vox;              // voxel points
    uint32_t* run;            // voxel run starts
    uint32_t *par, *cnt, *lab, *uk, *ca, *ord, *droot, *dsz, *rank, *fin, *off, *rk;
    uint32_t* cstart;         // dense neighbour grid: per-cell start in ord (LG_DCELLS_MAX + 2)
    uint32_t* hmeta;          // pinned host copy of the meta words (the one round trip per frame)
    uint32_t* hint;           // pinned host word (device address), or null: whether the last frame
                              // fit the LDS backend (LG_HINT_SMALL)
    uint32_t* cstat;          // per-chunk statistics [chunk][LG_CS_WORDS], reduced into meta by
                              // one workgroup (same-address atomics from every chunk serialise)
    uint32_t* pq;             // PCL voxel order: work queue of introsort ranges (lg_pcl_sort)
    uint32_t pq_cap;          //   entries
    uint64_t* pqst;           //   the partition levels' look-back words (tickets, finished, per tile),
                              //   two sets of pq_tmax + 2, then two sets of PQ_MAXR range counts
    uint32_t pq_tmax;         //   tiles a level can have (lg_pq_level)
    uint64_t* pqf;            //   the dataflow partition's queue (lg_pq_flow): counters, entries,
    uint32_t pqf_cap;         //   look-back, range and count words for pqf_cap tickets
    uint64_t* pqr;            //   the records beside the L and R lists (2 N words)
    uint32_t force_global;    // diagnostics: global backend even when M fits the LDS path
    uint32_t pcl_levels_cap;  // diagnostics: at most this many PCL partition levels (0: no cap)
    uint32_t force_wait_fail; // diagnostics (cg_debug_route 10): the first partition level reports
                              // a timed-out wait, as if its range never completed
    uint32_t pidx_base;       // frame index of the first point at L.in (a tile of a larger frame)
};
// Bytes of the large-frame scratch for frames of n points, and its layout at base.
uint64_t cg_large_bytes(uint32_t n_points);
uint32_t cg_large_pq_words();   // words of the PCL sort's range lists (diagnostics)
void cg_large_layout(uint8_t* base, uint32_t n_points, LgScratch& S);
// Run n_frames frames of more than CG_MAX_POINTS points, one at a time. Frames of up to
// LG_DEV_MAX_POINTS points in pipeline or detect mode with PCL's voxel order are sized on the
// device (every launch from N, counts read where they are used): enqueued without a host round
// trip, and replayed from a captured hipGraph per (frame, arguments) when `graphs` is given.
// Other frames synchronise s once per frame (the survivor count sizes the backend).
// (PCL's order keeps at most PQ_MAXR ranges per partition level: 4M detector points)
#define LG_DEV_MAX_POINTS (1u << 22)
struct LgGraphs;   // cg_large.hip: the handle's captured per-frame graphs
void cg_large_graphs_free(LgGraphs* g);
// The hint word (LgScratch::hint, pinned; the host reads it without synchronising, so it may
// come from an earlier frame: either value gives exact results, only the launch count varies):
enum {
    LG_HINT_SMALL = 0,    // 1 + (the last frame's detector input fit the LDS backend)
    LG_HINT_WORDS = 1
};
// hint: the LG_HINT_WORDS words as read (null: none). After a large frame the LDS backend's
// launch is left out (a small frame then takes the global backend).
int cg_run_large(const CgLaunch& L, const CgDevParams& P, int kmode, LgScratch S, hipStream_t s,
                 const LgScratch* S2 = nullptr, LgGraphs** graphs = nullptr, const uint32_t* hint = nullptr);
// The phases of cg_run_large for one frame f (also the tiles of cg_tile_*):
//   front: meta init + pass 1 (ground-only mode: the whole ground output);
//   decide: thresholds from meta, pass 2, candidates -> survivors (pipeline mode);
//   backend: detector backend over meta[LG_MS] survivors + npad pads, header N = n_total, K.
// szfl: 0, or (cg_run_large's device-sized backend) LG_SZ_ON | flags: the decisions' fold also
// writes the detector input's size and backend (LG_MALL ... LG_SMALL).
int cg_large_front(const CgLaunch& L, const CgDevParams& P, int kmode, LgScratch S, hipStream_t s, uint32_t f,
                   bool init, uint32_t szfl = 0);
int cg_large_decide(const CgLaunch& L, const CgDevParams& P, LgScratch S, hipStream_t s, uint32_t f,
                    uint32_t szfl = 0);
#define CG_K_FROM_META 0xffffffffu   // cg_large_backend: read K from the frame's meta words
int cg_large_backend(const CgLaunch& L, const CgDevParams& P, int kmode, LgScratch S, hipStream_t s, uint32_t f,
                     uint32_t n_total, uint32_t K);
// A tiled frame's gathered survivors and merged counts (K, Ms, nfin, bounds keys) into S.
// The 9 tile counts (cg_tile_decide's layout) from the meta words to d_counts, on stream s.
int cg_large_tile_counts(LgScratch S, uint32_t* d_counts, hipStream_t s);
int cg_large_set_survivors(LgScratch S, const CgDevParams& P, const float* d_points, const uint32_t* d_index,
                           uint32_t n, const uint32_t* counts, hipStream_t s);
// C5 halo tiling (cg_large.hip): a slab's voxels and components -> records; cross-slab
// edges -> component pairs (count at d_count); the merge of all slabs -> results in slot 0.
int cg_halo_local_run(const CgLaunch& L, const CgDevParams& P, LgScratch S, hipStream_t s, const float* d_points,
                      const uint32_t* d_index, uint32_t n, uint32_t npad_local, uint32_t npad_all,
                      const uint32_t* counts, uint32_t N, uint32_t key_bits, uint32_t* d_rec, uint32_t cap,
                      uint32_t* n_vox);
int cg_halo_edges_run(const uint32_t* own, uint32_t n_own, const uint32_t* halo, uint32_t n_halo, float r2,
                      uint32_t* pairs, uint32_t cap, uint32_t* d_count, hipStream_t s);
int cg_halo_merge_run(const CgLaunch& L, const CgDevParams& P, LgScratch S, hipStream_t s, const uint32_t* d_rec,
                      uint32_t V, const uint32_t* d_pairs, uint32_t np, uint32_t key_bits, uint32_t Mtot,
                      uint32_t K);
void cg_halo_plan_compute(const CgDevParams& P, const uint32_t* merged_counts, uint32_t N, uint32_t n_ranks,
                          struct cg_halo_plan* out);
int cg_launch_halo_owner(const float* pts, uint32_t n, float inv0, int32_t min_b0, uint32_t slab_w, uint32_t slabs,
                         int32_t* out, hipStream_t s);
// The LDS backend of the frame kernel on a large frame's survivors (M <= CG_MMAX).
int cg_launch_lg_back_small(const CgLaunch& L, const CgDevParams& P, const LgScratch& S, uint32_t f,
                            uint32_t npad, uint32_t K, hipStream_t s);

// Bytes of HBM scratch one frame of n points needs for the global (non-LDS) path.
uint64_t cg_scratch_bytes(uint32_t n_points);
// Enqueue the batch kernel (one fused workgroup per frame). Returns a hipError_t.
int cg_launch_batch(const CgLaunch& L, const CgDevParams& P, int kmode, hipStream_t s);
// Cone re-crop (cg_recrop.hip): exact float form of the reference's double box compares.
struct RcBox { float lox, hix, loy, hiy; };
#define CG_RECROP_MAX_BOXES 256   // boxes per launch (more: several launches)
uint32_t cg_recrop_blocks(uint32_t n_points);
// write = false: cnt[b * blocks + blk] = points of block blk in box b; write = true: out at
// off[b * blocks + blk] + in-block rank. pipeline: only groundless-cloud points (d_seckeys =
// the frame's 18 sector-minimum keys).
int cg_launch_recrop(const CgLaunch& L, const CgDevParams& P, bool pipeline, const uint32_t* d_seckeys,
                     const RcBox* d_boxes, uint32_t nb, uint32_t* d_cnt, const uint32_t* d_off, float4* d_out,
                     bool write, hipStream_t s);

// One frame's results packed for one device-to-host copy (word offsets; entries beyond
// CG_PACK_MAX are fetched separately).
#define CG_PACK_MAX 1024
#define CG_PACK_VOX CG_HDR_WORDS
// (header word CG_HDR_ERR of a large frame whose device-side wait gave up, LG_PQ_TIMEOUT:
// CG_HDR_E_WAIT, include/cones_gpu.h)
#define CG_PACK_LAB (CG_PACK_VOX + 4 * CG_PACK_MAX)
#define CG_PACK_OFFS (CG_PACK_LAB + CG_PACK_MAX)
#define CG_PACK_IDX (CG_PACK_OFFS + CG_PACK_MAX + 1)
#define CG_PACK_CEN (CG_PACK_IDX + CG_PACK_MAX)
#define CG_PACK_DONE (CG_PACK_CEN + 2 * CG_PACK_MAX)
#define CG_PACK_WORDS (CG_PACK_DONE + 1)
int cg_launch_pack(const CgLaunch& L, uint32_t f, uint32_t* out, hipStream_t s);
// Colour classifier (cg_colornet.hip): one workgroup per cone cloud.
int cg_launch_colornet(const float4* pts, const uint32_t* offs, uint32_t n_cones, const float* w, int32_t* colors,
                       float* probs, uint8_t* images, hipStream_t s);
int cg_launch_selftest_atan2f(const float* y, const float* x, float* out, uint32_t n, hipStream_t s);
int cg_launch_selftest_sqrt(const double* in, double* out, uint32_t n, hipStream_t s);
