// lgm_amd/csrc/common.h -- shared host-side helpers of liblgm_amd.so: thread-local error string, launch checks,
// and the per-call diagnostics (include/lgm_common.h lgm_diag: the HIP-event kernel profiler bench.py uses to time
// each kernel on the stream it is launched on).
#pragma once
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "lgm_common.h"

namespace lgm {

void set_error(const char *fmt, ...);
void clear_error();

// The diagnostics of the entry point running on this thread: set for the duration of one call by a DiagScope at
// its top (entry points run synchronously on the caller's thread and enqueue everything before returning), so
// nothing outlives the call.
struct DiagScope {
    explicit DiagScope(const lgm_diag *d);
    ~DiagScope();
    DiagScope(const DiagScope &) = delete;
    DiagScope &operator=(const DiagScope &) = delete;
};
const lgm_diag *call_diag();

// Kernel timing hooks: no-ops unless the current call has a profiler.
void prof_begin(const char *name, hipStream_t st);
void prof_end(hipStream_t st);

}  // namespace lgm

#define LGM_LAUNCH_CHECK(name)                                                                                 \
    do {                                                                                                       \
        hipError_t e_ = hipGetLastError();                                                                     \
        if (e_ != hipSuccess) {                                                                                \
            lgm::set_error("%s launch failed: %s", name, hipGetErrorString(e_));                               \
            return LGM_E_HIP;                                                                                  \
        }                                                                                                      \
    } while (0)

// Launch `stmt` (a kernel launch on stream st) bracketed by profiler events and checked.
#define LGM_LAUNCH(name, st, stmt)                                                                             \
    do {                                                                                                       \
        lgm::prof_begin(name, st);                                                                             \
        stmt;                                                                                                  \
        lgm::prof_end(st);                                                                                     \
        LGM_LAUNCH_CHECK(name);                                                                                \
    } while (0)
