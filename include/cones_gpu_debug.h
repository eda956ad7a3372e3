/* cones_gpu_debug.h — test and diagnostic entry points of libcones_gpu.so.
 *
 * NOT part of the product boundary: a ROS integrator includes only cones_gpu.h. These calls
 * exist for the repository's own tests, bench and profiling tools (device self-checks of the
 * exact libm restatements, per-phase timestamps, launch spans, forced routes that inject the
 * failures the product must survive, raw scratch dumps). They are exported by the same library
 * so that the tests exercise the shipped code object, and they may change without an ABI bump.
 */
#ifndef CONES_GPU_DEBUG_H
#define CONES_GPU_DEBUG_H
#include "cones_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- device self-checks (tests) ------------------------------------------------------ */
/* Evaluate the device atan2f / sector / sqrt restatements on n host inputs (device round
 * trip), for comparison with the host libm in tests. atan2f: out[2i] = the exact restatement,
 * out[2i+1] = sector + 32 * (angle filter at ang_hi = 1.3 removes it), both through the
 * certified fast classification. */
int cg_selftest_atan2f(cg_handle* h, const float* y, const float* x, float* out, uint32_t n);
int cg_selftest_sqrt(cg_handle* h, const double* s, double* out, uint32_t n);

/* Diagnostics: per-workgroup phase timestamps (s_memrealtime, 100 MHz; 32 slots per frame) for the
 * next batch calls; enable = 0 frees the buffer. Fetch synchronises the batch stream. */
int cg_debug_stamps(cg_handle* h, int enable);
/* Timing: the next cg_run_batch launch of the frame kernel records its execution span in
 * d_span (device memory, CG_SPAN_WORDS x uint64 the caller sets to {UINT64_MAX, 0, 0, 0}):
 * [0] the first workgroup's start and [1] the last workgroup's end, s_memrealtime ticks
 * (100 MHz); [2] the sum over workgroups of their shader cycles (s_memtime) and [3] of their
 * s_memrealtime ticks, so [2] / [3] x 100 MHz is the shader clock the launch ran at. Atomics by
 * one lane per workgroup at each end; frames of more than 65,536 points (large-frame path) do
 * not record. */
#define CG_SPAN_WORDS 4
int cg_debug_launch_span(cg_handle* h, void* d_span);
/* The same for the handle's next n_launches batch launches, launch k into
 * d_spans[CG_SPAN_WORDS k, CG_SPAN_WORDS (k + 1)) (no host call between the launches). */
int cg_debug_launch_spans(cg_handle* h, void* d_spans, uint32_t n_launches);
int cg_debug_stamps_fetch(cg_handle* h, uint64_t* out, uint32_t n_frames);

/* Diagnostics: route every frame through the large-frame path (1), and also through its
 * global HBM backend even when the detector input fits the LDS backend (2); run single-frame
 * calls in one workgroup instead of the per-chunk split launch (3), or split with the input
 * copied by DMA instead of read by the kernel from pinned memory (4); the global backend with
 * the PCL voxel sort cut after one partition level, so its leaves longer than the LDS leaf
 * are finished in HBM side by side (5); single-frame calls whose staged chunks are never
 * published, so every chunk workgroup times out and the call re-runs the frame by DMA (6,
 * tests of that retry); single-frame split calls whose chunk workgroup 0 gives up waiting for
 * the other chunks at once, so the call re-runs the frame in one workgroup (9, tests of that
 * retry); large frames whose PCL-order partition gives up waiting on its first range (10, tests
 * of that failure: the range's tiles take the expired-wait path itself, store their records
 * unchanged and queue the range whole as a leaf, and the fetch fails with CG_E_DEVICE). Route 10
 * acts only where that partition runs: device-sized frames (65,536 < N <= 2^22 points, pipeline
 * or detect mode, PCL voxel order) whose index_vector holds more than 2,048 records; the flag is
 * read by the clustering tail of that path, which every such frame runs; 0 = automatic. */
int cg_debug_route(cg_handle* h, int route);
/* Diagnostics: the meta words of the last large frame (sector minimum keys 0-17, touched
 * bins 18, K 19, candidates 20, survivors 21, ...; cg_internal.h LG_*). */
int cg_debug_large_meta(cg_handle* h, uint32_t* out, uint32_t n_words);
/* Diagnostics: raw large-frame scratch of the last frame: 0 = meta words, 1 = z codes
 * ([chunk][group][lane] words of 8 codes), 2 = ground-mode kept bits, 3 = the PCL voxel sort's
 * range lists (8 header words: level counts, leaf count; then 4 lists of 5-word entries),
 * 4 = the first 1024 bytes of the radix histogram area (phase stamps of variant builds). */
int cg_debug_large_buffer(cg_handle* h, int which, void* out, uint64_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* CONES_GPU_DEBUG_H */
