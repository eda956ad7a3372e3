// Variant build: lg_pq_flow's per-ticket record (entry taken, split done, range word complete,
// end, the entry's words) into the large scratch's histogram area from word 128 (free in the
// device-sized path), read with cg_debug_large_buffer(h, 4, ...) (tools/pqf_stamps.py).
//   VARIANT=tools/variants/pqf_stamps.h API_FLAGS=-DCG_DEBUG_HIST_BYTES=262144 tools/build_variant.sh pqfst
#define CG_DEBUG_HIST_BYTES 262144
#define CG_HOOK_PQF(S, t, k, v)                                                              \
    do {                                                                                     \
        if ((t) < 4000u) ((unsigned long long*)(S).hist)[128 + 6ull * (t) + (k)] = (v);      \
    } while (0)
