"""Builds the in-tree HIP library lgm_amd/_lib/liblgm_amd.so for gfx950 with hipcc (no JIT cache, no torch
C++ ABI: the library exports a plain C ABI, include/*.h). Run: python -m lgm_amd.build"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SOURCES = ["csrc/common.hip", "csrc/render_bin.hip", "csrc/render_raster.hip", "csrc/render_api.hip",
           "csrc/attention.hip", "csrc/head.hip", "csrc/mvattn.hip", "csrc/wgrad.hip"]
# per-source extra flags. attention.hip: no NaN semantics -- its max / exp chains then skip the quieting
# canonicalisations clang inserts before every fmaxf of an MFMA result (the render kernels keep IEEE NaN handling:
# degenerate-Gaussian tests such as !(det > 0) rely on it)
FILE_FLAGS = {"csrc/attention.hip": ["-fno-honor-nans"]}
OUT = os.path.join(HERE, "_lib", "liblgm_amd.so")
ARCH = os.environ.get("LGM_AMD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def sources():
    return [os.path.join(HERE, s) for s in SOURCES if os.path.exists(os.path.join(HERE, s))]


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = sources() + [os.path.join(ROOT, "include", f) for f in os.listdir(os.path.join(ROOT, "include"))] + \
        [os.path.join(HERE, "csrc", f) for f in os.listdir(os.path.join(HERE, "csrc")) if f.endswith(".h")]
    return any(os.path.getmtime(p) > t for p in deps)


def build(force: bool = False, verbose: bool = False, out: str = None, defines=()) -> str:
    """Compile every source and link the shared library (`out` and `defines` build A/B variants)."""
    out = out or OUT
    if out == OUT and not force and not needs_build():
        return OUT
    os.makedirs(os.path.dirname(out), exist_ok=True)
    objs, cmds = [], []
    tag = "" if out == OUT else "." + os.path.basename(out)
    for src in sources():
        obj = os.path.join(HERE, "_lib", os.path.basename(src) + tag + ".o")
        extra = FILE_FLAGS.get(os.path.relpath(src, HERE), [])
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
               "-munsafe-fp-atomics", "-fno-slp-vectorize", "-I", os.path.join(ROOT, "include"), "-I",
               os.path.join(HERE, "csrc"), "-c", src, "-o", obj] + extra + \
            [d if d.startswith("-") else f"-D{d}" for d in defines]  # A/B variants: defines or extra flags
        if verbose:
            print(" ".join(cmd))
        cmds.append(cmd)
        objs.append(obj)
    # the sources compile independently: in parallel (at most 8 at once: the container and the GPU box's share)
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=min(8, len(cmds))) as ex:
        for r in list(ex.map(lambda c: subprocess.run(c), cmds)):
            if r.returncode:
                raise subprocess.CalledProcessError(r.returncode, r.args)
    tmp = out + ".tmp"
    subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs, check=True)
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
