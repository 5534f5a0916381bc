/*
 * lgm_common.h -- C ABI shared by the render, head and attention entry points of liblgm_amd.so:
 * error reporting and the optional per-call diagnostics (a kernel profiler: HIP events recorded on the caller's
 * stream around every kernel the call launches; and the render kernels' device work counters). There is no
 * reference counterpart: the reference has no profiling hooks beyond the CUDA-event FPS label of gui.py:59-104
 *  and the EXT rasterizer's `debug` flag (core/gs.py:70); bench.py uses the profiler to time the
 * dominant kernel live inside its measured steps.
 *
 * State: the library keeps NO mutable global state besides the thread-local error string. Diagnostics are
 * per call: every compute entry point takes a trailing `const lgm_diag *diag` (NULL = none) that applies to the
 * kernels of that call only.
 */
#ifndef LGM_COMMON_H
#define LGM_COMMON_H
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

#define LGM_OK 0
#define LGM_E_INVALID -1   /* bad sizes / null pointers */
#define LGM_E_WORKSPACE -2 /* workspace too small */
#define LGM_E_HIP -3       /* a HIP call or launch failed */

/* Thread-local description of the last error ("" if none). */
const char *lgm_last_error(void);

/* ABI version (bumped on any signature change). 3: per-call lgm_diag, LGM_RENDER_NO_CULL as a per-call option.
 * 4: lgm_diag.det_limit_log2. 5: lgm_attn_workspace_size takes D. */
int lgm_abi_version(void);

/* Profiler object: create, read per-kernel totals, reset, destroy. It records into itself only while a call is
 * given it through lgm_diag.profiler (a profiler may be shared by calls on several threads: it locks).
 * lgm_profiler_summary synchronises on the recorded events and writes lines "name count total_ms\n". */
typedef struct lgm_profiler lgm_profiler;
lgm_profiler *lgm_profiler_create(void);
int lgm_profiler_summary(lgm_profiler *p, char *buf, size_t len);
int lgm_profiler_reset(lgm_profiler *p);
void lgm_profiler_destroy(lgm_profiler *p);

/* Per-call diagnostics (all fields optional). */
typedef struct lgm_diag {
    lgm_profiler *profiler;              /* HIP events around every kernel of the call, or NULL */
    unsigned long long *render_counters; /* DEVICE work counters of the render kernels (see lgm_render.h), or NULL */
    int det_limit_log2;                  /* test hook, 0 = none: LGM_RENDER_DETERMINISTIC's per-flush overflow bound
                                            becomes 2^det_limit_log2 instead of 2^62 / 2^ceil(log2 tiles), so a test
                                            can force the saturation path (gradients poisoned with NaN) */
} lgm_diag;

#ifdef __cplusplus
}
#endif
#endif
