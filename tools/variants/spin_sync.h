// Variant build (tools/build_variant.sh): the host busy-polls hipStreamQuery instead of the
// blocking hipStreamSynchronize (a host core for the wake-up latency).
//   VARIANT=tools/variants/spin_sync.h tools/build_variant.sh spin
#include <hip/hip_runtime.h>
static inline hipError_t cg_variant_spin_wait(hipStream_t s) {
    hipError_t e;
    while ((e = hipStreamQuery(s)) == hipErrorNotReady) {
    }
    (void)hipGetLastError();   // the polls' not-ready status is not an error
    return e;
}
#define CG_HOOK_STREAM_WAIT(s) cg_variant_spin_wait(s)
