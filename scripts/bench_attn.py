"""Attention micro-bench at LGM's MVAttention shapes.

For each level: the HIP kernels (lgm_amd.attention.packed_attention) fwd and fwd+bwd in TFLOP/s, plus
torch.nn.functional.scaled_dot_product_attention on the same tensors as a comparator (the ROCm flash backend
torch ships; the reference's xformers kernel is CUDA-only). FLOPs: fwd 4 B H L^2 D, bwd 10 B H L^2 D (S recompute,
dP, dV, dQ, dK). Prints one JSON line per shape and a summary of per-kernel HIP-event times.
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lgm_amd import _native  # noqa: E402
from lgm_amd.dist import warm_up  # noqa: E402
from lgm_amd.attention import packed_attention  # noqa: E402

# (name, B objects, views F, tokens per view h*w, heads, head dim)
LEVELS = [
    ("big256_c512_32x32", 8, 4, 32 * 32, 16, 32),
    ("big256_c1024_16x16", 8, 4, 16 * 16, 16, 64),
    ("big256_c1024_8x8", 8, 4, 8 * 8, 16, 64),
    ("cfg4_c512_40x40", 1, 6, 40 * 40, 16, 32),
    ("cfg4_c1024_20x20", 1, 6, 20 * 20, 16, 64),
]


def timed(fn, iters):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    warm_up(fn, 1, torch.cuda.synchronize)  # >= 50 ms: the GPU clocks' ramp (lgm_amd/dist.py)
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f16", "f32"])
    ap.add_argument("--no-sdpa", action="store_true")
    args = ap.parse_args()
    dt = {"bf16": torch.bfloat16, "f16": torch.float16, "f32": torch.float32}[args.dtype]
    dev = torch.device("cuda:0")
    prof = _native.KernelProfiler()
    for name, B, Fv, hw, H, D in LEVELS:
        L = Fv * hw
        qkv = torch.randn(B, L, 3, H, D, device=dev, dtype=dt)
        d_o = torch.randn(B, L, H, D, device=dev, dtype=dt)
        x = qkv.clone().requires_grad_(True)
        fl_f = 4.0 * B * H * L * L * D
        fl_b = 10.0 * B * H * L * L * D

        def ours_f():
            with torch.no_grad():
                packed_attention(qkv)

        def ours_fb():
            x.grad = None
            packed_attention(x).backward(d_o)

        t_f = timed(ours_f, args.iters)
        prof.reset()
        with prof:
            t_fb = timed(ours_fb, args.iters)
        ks = prof.summary()
        rec = {"level": name, "B": B, "L": L, "H": H, "D": D, "dtype": args.dtype,
               "fwd_ms": t_f, "fwd_tflops": fl_f / t_f / 1e9, "fwdbwd_ms": t_fb,
               "fwdbwd_tflops": (fl_f + fl_b) / t_fb / 1e9,
               "kernels_ms": {k: v[1] / v[0] for k, v in ks.items()}}
        if not args.no_sdpa:
            qs, ks_, vs = (qkv[:, :, i].transpose(1, 2) for i in range(3))
            xs = [t.detach().clone().requires_grad_(True) for t in (qs, ks_, vs)]
            dos = d_o.transpose(1, 2)

            def sd_f():
                with torch.no_grad():
                    F.scaled_dot_product_attention(qs, ks_, vs)

            def sd_fb():
                for t in xs:
                    t.grad = None
                F.scaled_dot_product_attention(*xs).backward(dos)

            try:
                rec["sdpa_fwd_ms"] = timed(sd_f, args.iters)
                rec["sdpa_fwdbwd_ms"] = timed(sd_fb, args.iters)
                rec["sdpa_fwd_tflops"] = fl_f / rec["sdpa_fwd_ms"] / 1e9
                rec["sdpa_fwdbwd_tflops"] = (fl_f + fl_b) / rec["sdpa_fwdbwd_ms"] / 1e9
            except RuntimeError as e:  # backend unavailable for this shape/dtype
                rec["sdpa_error"] = str(e)[:200]
        print(json.dumps(rec), flush=True)
        del qkv, d_o, x
        torch.cuda.empty_cache()
    prof.close()


if __name__ == "__main__":
    main()
