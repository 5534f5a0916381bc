"""The C-ABI library loads and exports every symbol declared in include/*.h (no GPU compute here)."""
import ctypes
import glob
import os
import re

from lgm_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        txt = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        syms |= set(re.findall(r"\b(lgm_[a-z0-9_]+)\s*\(", txt))
    return syms


def test_library_exports_all_declared_symbols():
    from lgm_amd import build as B
    B.build()
    L = ctypes.CDLL(_native.LIB_PATH)
    syms = declared_symbols()
    assert "lgm_render_forward" in syms and "lgm_render_backward" in syms
    missing = [s for s in sorted(syms) if not hasattr(L, s)]
    assert not missing, missing
    # every declared symbol has a Python binding signature
    assert not [s for s in syms if s not in _native.SIGNATURES], [s for s in syms if s not in _native.SIGNATURES]


def test_workspace_and_errors():
    L = _native.lib()
    assert L.lgm_abi_version() == _native.ABI_VERSION
    w1 = L.lgm_render_workspace_size(1, 6, 100000, 256, 256, 0)
    w2 = L.lgm_render_workspace_size(1, 6, 100000, 256, 256, 1000000)
    assert w1 > w2 > 0
    assert L.lgm_render_workspace_size(0, 6, 10, 256, 256, 0) == 0
    # invalid arguments are reported, never thrown
    rc = L.lgm_render_forward(1, 1, 10, 16, 16, None, None, None, None, 1.0, 1.0, 1.0, None, None, None, None, None,
                              0, 0, None, 0, None, None)
    assert rc < 0 and b"null" in L.lgm_last_error()
    # attention: unsupported head dim / dtype are reported, never thrown
    rc = L.lgm_attn_forward(1, 1, 16, 2, 48, 0.1, None, None, None, 0, None, None, None, None)
    assert rc < 0 and b"D must be" in L.lgm_last_error()
    assert L.lgm_attn_workspace_size(0, 2, 100, 4, 32) == 2 * 100 * 4 * 4  # fp32: delta
    assert L.lgm_attn_workspace_size(1, 2, 100, 4, 32) >= 2 * 100 * 4 * (4 + 2 * 32)  # bf16: delta + Q * c


def test_no_process_wide_switches():
    """no global mutable state besides the error string. The round-2 process-wide setters
    (lgm_render_set_flags, lgm_render_debug_counters, lgm_profiler_attach) are gone: NO_CULL is a per-call option
    bit and diagnostics a per-call lgm_diag; every compute entry point that takes a stream takes a diag after it
    (the three workspace-inspection copies excepted)."""
    from lgm_amd import build as B
    B.build()
    L = ctypes.CDLL(_native.LIB_PATH)
    for gone in ("lgm_render_set_flags", "lgm_render_debug_counters", "lgm_profiler_attach"):
        assert not hasattr(L, gone), gone
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        txt = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        for name, args in re.findall(r"\b(lgm_[a-z0-9_]+)\s*\(([^)]*)\)\s*;", txt):
            if "void *stream" in args and name not in ("lgm_render_tile_lists", "lgm_render_pixel_state",
                                                              "lgm_render_records", "lgm_render_needle_flags"):
                assert args.rstrip().endswith("const lgm_diag *diag"), name
