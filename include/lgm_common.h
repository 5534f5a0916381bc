/*
 * lgm_common.h -- C ABI shared by the render and attention entry points of liblgm_amd.so:
 * error reporting and an optional kernel profiler (HIP events recorded on the caller's stream around
 * every kernel the library launches). There is no reference counterpart: the reference has no profiling hooks
 * beyond the CUDA-event FPS label of gui.py:59-104; bench.py uses this to time the dominant
 * kernel live inside the timed region.
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

/* ABI version (bumped on any signature change). */
int lgm_abi_version(void);

/* Profiler: create, attach process-wide (NULL detaches; the only mutable global besides the per-thread error
 * string), read per-kernel totals, destroy.
 * lgm_profiler_summary synchronises on the recorded events and writes lines "name count total_ms\n". */
typedef struct lgm_profiler lgm_profiler;
lgm_profiler *lgm_profiler_create(void);
int lgm_profiler_attach(lgm_profiler *p);
int lgm_profiler_summary(lgm_profiler *p, char *buf, size_t len);
int lgm_profiler_reset(lgm_profiler *p);
void lgm_profiler_destroy(lgm_profiler *p);

#ifdef __cplusplus
}
#endif
#endif
