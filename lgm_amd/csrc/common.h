// lgm_amd/csrc/common.h -- shared host-side helpers of liblgm_amd.so: thread-local error string, launch checks,
// and the optional thread-local HIP-event kernel profiler (include/lgm_common.h) used by bench.py to time each
// kernel on the stream it is launched on.
#pragma once
#include <hip/hip_runtime.h>
#include <stdio.h>

namespace lgm {

void set_error(const char *fmt, ...);
void clear_error();

// Kernel timing hooks: no-ops unless a profiler is attached to the calling thread.
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
