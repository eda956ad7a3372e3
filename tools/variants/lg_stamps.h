// Variant build (tools/build_variant.sh): s_memrealtime stamps of lg_cluster_tail's phases into
// the first words of the large scratch's histogram area (free in the device-sized path), read
// with cg_debug_large_buffer(h, 4, ...) (tools/lg_stamps.py).
//   VARIANT=tools/variants/lg_stamps.h tools/build_variant.sh lgst
#define CG_HOOK_LG_STAMP(S, i)                                                                    \
    do {                                                                                          \
        if (threadIdx.x == 0) ((unsigned long long*)(S).hist)[i] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
