// Variant build (tools/build_variant.sh): the frame kernel returns after phase CG_EXP_STOP
// (1 pass 1, 2 pass 2 + survivor gather, 3 pads + bounds) with the frame's header zeroed, and
// still stamps its launch span. Measures what the tail after that phase costs.
//   VARIANT=tools/variants/exp_stop.h tools/build_variant.sh stop1 -DCG_EXP_STOP=1
// (translation units built without -DCG_EXP_STOP keep the product's hook)
#ifdef CG_EXP_STOP
#define CG_HOOK_FRAME_PHASE(k)                                                                          \
    if ((k) == CG_EXP_STOP) {                                                                           \
        if (tid == 0) { uint32_t* h_ = L.hdr + (uint64_t)f * 8; h_[0] = N; h_[1] = h_[2] = h_[3] = h_[4] = h_[5] = 0; } \
        if (L.span && tid == 0) atomicMax(&L.span[1], (unsigned long long)__builtin_amdgcn_s_memrealtime()); \
        return;                                                                                         \
    }
#endif
