// cg_host.h — host-only helpers of the C-ABI (cg_host.cpp): no HIP runtime calls, so they
// also build under the host sanitizers. Not part of the public boundary.
#pragma once
#include <cstdarg>
#include <stdint.h>
#include "../../include/cones_gpu.h"
#include "cg_internal.h"

// Sets the thread-local message cg_last_error returns (printf format); returns code.
int cg_fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int cg_vfail(int code, const char* fmt, va_list ap);
// cg_params -> the device's exact thresholds (CG_E_INVALID for a bad leaf size)
int cg_prepare_params(const cg_params& p, CgDevParams& d);
// argument checks of the C-ABI entry points (CG_OK or an error code with the message set)
int cg_check_view(const cg_cloud_view* v);
int cg_check_tile(const cg_tile* t);
int cg_halo_counts_check(const uint32_t* merged_counts, uint32_t n_total);
int cg_halo_plan_check(const cg_halo_plan* p);
