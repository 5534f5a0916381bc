"""ctypes binding of the C ABI in include/lgm_render.h and include/lgm_attn.h (liblgm_amd.so).

There is no fallback: if the library is missing or cannot be loaded, every op raises. torch is imported first so
that the library's NEEDED libamdhip64.so.7 resolves to the HIP runtime torch already loaded (same soname), giving
one HIP runtime per process and letting device pointers and streams flow between torch and the library.

The library holds no mutable global state besides its thread-local error string: diagnostics (the kernel profiler,
the render work counters) travel with each call as an `lgm_diag` (include/lgm_common.h). The harness-side switch
for them is `diagnostics(...)` here, whose value every wrapper passes as the call's `diag` (None = NULL).
"""
from __future__ import annotations

import contextlib
import ctypes
import os

import torch  # noqa: F401  (must be loaded before the HIP library, see above)

LIB_PATH = os.environ.get("LGM_AMD_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib",
                                                          "liblgm_amd.so")

_c_int, _c_ll, _c_float, _c_size, _vp = ctypes.c_int, ctypes.c_longlong, ctypes.c_float, ctypes.c_size_t, ctypes.c_void_p

SIGNATURES = {
    "lgm_abi_version": (_c_int, []),
    "lgm_last_error": (ctypes.c_char_p, []),
    "lgm_render_workspace_size": (_c_size, [_c_int, _c_int, _c_int, _c_int, _c_int, _c_ll]),
    "lgm_render_workspace_size_opts": (_c_size, [_c_int, _c_int, _c_int, _c_int, _c_int, _c_ll, _c_int]),
    "lgm_render_count_pairs": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _c_float, _c_float,
                                        _c_float, _vp, _c_size, _vp, _vp, _vp]),
    "lgm_render_forward": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _c_float, _c_float,
                                    _c_float, _vp, _vp, _vp, _vp, _vp, _c_size, _c_ll, _vp, _c_int, _vp, _vp]),
    "lgm_render_backward": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _c_float, _c_float,
                                     _c_float, _vp, _vp, _vp, _vp, _vp, _vp, _c_size, _c_ll, _c_int, _vp, _vp]),
    "lgm_attn_forward": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _c_float, _vp, _vp, _vp, _c_ll, _vp, _vp,
                                  _vp, _vp]),
    "lgm_attn_backward": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _c_float, _vp, _vp, _vp, _c_ll, _vp, _vp,
                                   _vp, _vp, _vp, _vp, _c_ll, _vp, _c_size, _vp, _vp]),
    "lgm_attn_workspace_size": (_c_size, [_c_int, _c_int, _c_int, _c_int, _c_int]),
    "lgm_mva_workspace_size": (_c_size, [_c_int, _c_int, _c_int, _c_int, _c_int]),
    "lgm_mva_norm_tokens": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_float, _vp, _vp, _vp,
                                     _vp, _vp, _vp, _vp, _c_size, _vp, _vp]),
    "lgm_mva_tokens_out": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _c_float, _vp,
                                    _vp, _vp]),
    "lgm_mva_backward_workspace_size": (_c_size, [_c_int, _c_int, _c_int, _c_int, _c_int]),
    "lgm_mva_tokens_out_backward": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _c_float, _vp,
                                             _vp, _vp, _vp]),
    "lgm_mva_norm_tokens_backward": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp,
                                              _vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_size, _vp, _vp]),
    "lgm_render_forward_loss": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _c_float,
                                         _c_float, _c_float, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_size, _c_ll, _c_int,
                                         _vp, _vp]),
    "lgm_render_backward_loss": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _c_float,
                                          _c_float, _c_float, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_size, _c_ll,
                                          _c_int, _vp, _vp]),
    "lgm_render_tile_lists": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _vp, _c_size, _c_ll, _vp, _vp, _vp,
                                       _vp]),
    "lgm_render_pixel_state": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _vp, _c_size, _c_ll, _vp, _vp, _vp]),
    "lgm_render_records": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _vp, _c_size, _c_ll, _vp, _vp, _vp, _vp]),
    "lgm_render_needle_flags": (_c_int, [_c_ll, _vp, _vp, _vp]),
    "lgm_render_det_flush_limit_log2": (_c_int, [_c_int, _c_int, _c_int]),
    "lgm_gaussian_head_forward": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp, _vp,
                                           _c_size, _vp, _vp]),
    "lgm_gaussian_head_workspace_size": (_c_size, [_c_int, _c_int, _c_int, _c_int]),
    "lgm_gaussian_head_backward": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                            _vp, _vp, _c_size, _vp, _vp]),
    "lgm_linear_wgrad_workspace_size": (_c_size, [_c_int, _c_int, _c_int, _c_int]),
    "lgm_linear_wgrad": (_c_int, [_c_int, _c_int, _c_int, _c_int, _vp, _c_ll, _vp, _c_ll, _vp, _vp, _vp, _c_size,
                                  _vp, _vp]),
    "lgm_profiler_create": (_vp, []),
    "lgm_profiler_summary": (_c_int, [_vp, ctypes.c_char_p, _c_size]),
    "lgm_profiler_reset": (_c_int, [_vp]),
    "lgm_profiler_destroy": (None, [_vp]),
}

_lib = None


ABI_VERSION = 5
RENDER_NO_CULL = 1  # include/lgm_render.h LGM_RENDER_NO_CULL
RENDER_CLAMP_IMAGE = 2  # include/lgm_render.h LGM_RENDER_CLAMP_IMAGE
RENDER_BACKWARD_AGAIN = 4  # include/lgm_render.h LGM_RENDER_BACKWARD_AGAIN
RENDER_DETERMINISTIC = 16  # include/lgm_render.h LGM_RENDER_DETERMINISTIC


class NativeError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(f"lgm_amd native library not built ({LIB_PATH}); run `python -m lgm_amd.build`")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name, None)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
        if L.lgm_abi_version() != ABI_VERSION:
            raise NativeError(f"{LIB_PATH}: ABI {L.lgm_abi_version()} != {ABI_VERSION}; rebuild (python -m lgm_amd.build)")
        _lib = L
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().lgm_last_error()
        raise NativeError(f"{what} failed (rc={rc}): {msg.decode() if msg else ''}")


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_of(device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_device_tensor(t: torch.Tensor, name: str):
    if not t.is_cuda:
        raise NativeError(f"{name} must be a GPU tensor: lgm_amd has no CPU path (the reference's rasterizer is "
                          "GPU-only too, core/gs.py:20)")


class _Diag(ctypes.Structure):
    """include/lgm_common.h lgm_diag."""
    _fields_ = [("profiler", _vp), ("render_counters", _vp), ("det_limit_log2", ctypes.c_int)]


_diag_cur = None  # the lgm_diag every wrapper passes while a diagnostics() block is open (None: NULL)


def diag():
    """The `diag` argument for the next C-ABI call: NULL unless a diagnostics() block is open. (Harness state, not
    library state: autograd runs the backward on its own thread, so a thread-local switch would miss it.)"""
    return None if _diag_cur is None else ctypes.byref(_diag_cur)


@contextlib.contextmanager
def diagnostics(profiler=None, render_counters=None, det_limit_log2=0):
    """Inside the block, every liblgm_amd call made through this package carries these diagnostics: a
    KernelProfiler and/or a device uint64 tensor for the render work counters (include/lgm_render.h), and the
    deterministic mode's overflow-bound test hook (include/lgm_common.h)."""
    global _diag_cur
    prev = _diag_cur
    d = _Diag(profiler.h if profiler is not None else None,
              render_counters.data_ptr() if render_counters is not None else None, int(det_limit_log2))
    _diag_cur = d
    try:
        yield d
    finally:
        _diag_cur = prev


class KernelProfiler:
    """HIP events around every kernel liblgm_amd launches (on the launching stream) while the profiler is entered
    (`with prof:` = diagnostics(profiler=prof)). summary() -> {kernel: (launches, total_ms)}."""

    def __init__(self):
        self.h = lib().lgm_profiler_create()
        self._cm = None

    def __enter__(self):
        self._cm = diagnostics(profiler=self)
        self._cm.__enter__()
        return self

    def __exit__(self, *exc):
        cm, self._cm = self._cm, None
        return cm.__exit__(*exc)

    def reset(self):
        lib().lgm_profiler_reset(self.h)

    def summary(self):
        buf = ctypes.create_string_buffer(1 << 16)
        check(lib().lgm_profiler_summary(self.h, buf, len(buf)), "lgm_profiler_summary")
        out = {}
        for line in buf.value.decode().splitlines():
            name, n, ms = line.split()
            out[name] = (int(n), float(ms))
        return out

    def close(self):
        if self.h:
            lib().lgm_profiler_destroy(self.h)
            self.h = None
