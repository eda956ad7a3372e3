// scratch_probe.hip — the round-2 probe's shape, rebuilt for its code-object metadata
// (tests/test_isa.py::test_out_of_line_probe_needs_scratch; DESIGN.md "Lessons"): the
// single-wave cluster-order sort out of line, its per-lane record passed by reference. Device
// code object only; never run.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../cones_perception_amd/csrc/cg_sort.h"
// the single-wave cluster-order sort called out of line, its record (a VGPR of the caller) by reference
__device__ __noinline__ void sort_ool(uint32_t& v, int n) { cg_std_sort_wave32(v, n); }
__global__ __launch_bounds__(64) void probe(const uint32_t* in, uint32_t* out, int n) {
    uint32_t v = in[threadIdx.x];
    sort_ool(v, n);
    out[threadIdx.x] = v;
}
