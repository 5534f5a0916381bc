"""bench.py -- BASELINE.json metric: Mpixels/s of forward+backward Gaussian rasterization, 256^2, 100k Gaussians,
6 views (BASELINE config 3), on 1/2/4/8 MI355X.

A step = GaussianRenderer.render (core/gs.py:31-98 API: forward of all 6 views, clamp) + autograd backward to
dL/dgaussians [1,N,14] for fixed seeded upstream gradients. Weak scaling: every rank renders its OWN scene
(seed 1 + rank; scene-sharded, no data-path collective); value = total pixels of all ranks / max
rank time. Per-kernel durations come from HIP events recorded by liblgm_amd on the launch stream inside the timed
region (lgm_amd._native.KernelProfiler); `roofline` prices the dominant kernel with SURVEY.md §8(d)'s algorithmic
bytes. The CPU baseline (rank 0, N=1) is the oracle port (oracle/raster_oracle.c, OpenMP over views) on the same
scene for a bounded number of repetitions.

    python bench.py [--gpus N --steps K --warmup W]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA peak (no sparsity)
N_GAUSS, VIEWS, RES = 100_000, 6, 256


def kernel_bytes(N, V, K, P):
    """SURVEY.md §8(d) algorithmic bytes per launch (all V views of one scene): fwd = 56N + 60K + 20P,
    bwd = 112N + 84K + 28P per view, K = upstream's num_rendered (summed over views here) even though fewer pairs
    are binned after exact culling (a build that culls more is still credited with K_ref).
    k_bin (preprocess + emit) carries 56N + 8K per view, k_sort 8K."""
    return {
        "k_bin": 56 * N * V + 8 * K,
        "k_sort": 8 * K,
        "k_render_fwd": 44 * K + 20 * P * V,
        "k_render_bwd": 84 * K + 28 * P * V,
        "k_preproc_bwd": 112 * N * V,
    }


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed PMC profile of this workload (rocprofv3 FETCH_SIZE x 2 +
    WRITE_SIZE, gfx950-corrected, scripts/gpu_pmc.sh -> scripts/pmc_summary.py --json), or null."""
    path = os.path.join(ROOT, "profiles", "pmc_latest.json")
    try:
        d = json.load(open(path))
        rec = d[kernel]
        return {"traffic": int(rec["hbm_read_bytes"] + rec["hbm_write_bytes"]),
                "traffic_source": f"profiles/pmc_latest.json (PMC passes at commit {d['_meta'].get('commit', '?')})"}
    except (OSError, KeyError, ValueError):
        return {"traffic": None}


def cpu_baseline(g, cv, cvp, tan, bg, d_img, d_alpha, seconds):
    from oracle import oracle as O
    O.build()
    threads = min(os.cpu_count() or 1, VIEWS)
    args = (g.numpy(), cv.numpy(), cvp.numpy(), tan, RES, RES, bg.numpy())
    kw = dict(d_image=d_img.numpy(), d_alpha=d_alpha.numpy(), nthreads=threads)
    O.render(*args, **kw)  # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        O.render(*args, **kw)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": round(reps * VIEWS * RES * RES / el / 1e6, 3), "unit": "Mpixels/s", "cores": threads,
            "kind": "port",
            "sample": f"oracle/raster_oracle.c fwd+bwd of the rank-0 cfg3 scene (100k Gaussians x 6 views x 256^2), "
                      f"{reps} repetitions in {el:.1f} s, OpenMP over views"}


def attention_bench(dev, steps: int = 10):
    """Secondary object: LGM's heaviest MVAttention level (core/unet.py:35-49 at C=512, 32x32, 4 views -> L = 4096
    tokens, 16 heads, D = 32; 8 objects per GPU as in the 'big' training batch), bf16 fwd+bwd through the HIP
    kernels (lgm_amd/attention.py), with torch's SDPA on the same tensors as a comparator. FLOPs 14 B H L^2 D."""
    import torch
    import torch.nn.functional as F

    from lgm_amd import _native
    from lgm_amd.attention import packed_attention
    B, L, H, D = 8, 4096, 16, 32
    g = torch.Generator(device="cpu").manual_seed(7)
    qkv = torch.randn((B, L, 3, H, D), generator=g).to(dev, torch.bfloat16)
    d_o = torch.randn((B, L, H, D), generator=g).to(dev, torch.bfloat16)
    x = qkv.clone().requires_grad_(True)

    def step():
        x.grad = None
        packed_attention(x).backward(d_o)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(steps):
            fn()
        en.record()
        torch.cuda.synchronize()
        return st.elapsed_time(en) / steps

    ms = timed(step)
    prof = _native.KernelProfiler()  # per-kernel times from a separate pass
    with prof:
        timed(step)
    kern = prof.summary()
    prof.close()
    qs, ks, vs = (qkv[:, :, i].transpose(1, 2).detach().clone().requires_grad_(True) for i in range(3))
    dos = d_o.transpose(1, 2)

    def sdpa():
        for t in (qs, ks, vs):
            t.grad = None
        F.scaled_dot_product_attention(qs, ks, vs).backward(dos)

    try:
        ms_sdpa = timed(sdpa)
    except RuntimeError:
        ms_sdpa = None
    flops = 14.0 * B * H * L * L * D
    tf = flops / ms / 1e9
    return {"workload": "MVAttention C=512 32x32 x 4 views (L=4096, 16 heads, D=32), 8 objects, fwd+bwd",
            "dtype": "bf16", "ms_per_step": round(ms, 4), "tflops": round(tf, 1),
            "roofline": {"bound": "mfma", "achieved": round(tf, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(tf / PEAK_BF16_TFLOPS, 4)},
            "kernels": {k: {"avg_us": round(1e3 * v / n, 2), "launches": n} for k, (n, v) in kern.items()},
            "torch_sdpa_tflops": round(flops / ms_sdpa / 1e9, 1) if ms_sdpa else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-attention", action="store_true", help="skip the secondary attention measurement")
    args = ap.parse_args()

    import torch

    from lgm_amd import dist as D
    info = D.rank_info()
    rank, world = info.rank, info.world
    torch.cuda.set_device(info.local)
    dev = torch.device("cuda", info.local)
    D.init("nccl", info, dev)

    from lgm_amd import GaussianRenderer, Options, _native
    from lgm_amd.cameras import orbit_cameras
    from lgm_amd.gs import count_pairs
    from lgm_amd.synthetic import synthetic_gaussians, synthetic_upstream_grads

    seed = D.scene_seed(rank)
    g_cpu = synthetic_gaussians(1, N_GAUSS, seed=seed)
    cv, cvp, cp = orbit_cameras(VIEWS)
    d_img, _, d_alpha, bg = synthetic_upstream_grads(1, VIEWS, RES, RES, seed=seed + 1000)
    renderer = GaussianRenderer(Options(output_size=RES))
    g = g_cpu.to(dev).requires_grad_(True)
    cvd, cvpd, cpd = cv[None].to(dev), cvp[None].to(dev), cp[None].to(dev)
    bgd, d_imgd, d_alphad = bg.to(dev), d_img.to(dev), d_alpha.to(dev)
    tan = float(renderer.tan_half_fov)
    K_binned, K = count_pairs(g.detach(), cvd, cvpd, tan, tan, RES, RES)

    def step():
        out = renderer.render(g, cvd, cvpd, cpd, bg_color=bgd)
        torch.autograd.backward([out["image"], out["alpha"]], [d_imgd, d_alphad])
        g.grad = None

    for _ in range(args.warmup):
        step()
    # the timed steps run with nothing attached; per-kernel HIP-event times come from a second, untimed pass of
    # the same K steps (the event records add marker packets between launches)
    el = D.timed_steps(step, args.steps, info, torch.cuda.synchronize, dev)
    prof = _native.KernelProfiler()
    with prof:
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
    kern = prof.summary()
    prof.close()

    P = RES * RES
    pixels = world * VIEWS * P * args.steps
    value = pixels / el / 1e6
    kb = kernel_bytes(N_GAUSS, VIEWS, K, P)
    per_kernel = {k: {"avg_us": round(1e3 * ms / n, 2), "launches": n} for k, (n, ms) in kern.items()}
    dom = max(kern.items(), key=lambda kv: kv[1][1])[0]
    dom_avg_s = kern[dom][1] / kern[dom][0] / 1e3
    achieved = kb.get(dom, 0) / dom_avg_s / 1e9
    step_bytes = sum(kb.values())
    ms_step = 1e3 * el / args.steps
    result = {
        "metric": "Mpixels/s fwd+bwd Gaussian raster (256^2, 100k gauss, 6 views)",
        "value": round(value, 2),
        "unit": "Mpixels/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (SURVEY.md 8(d): raw~N(0,1) through LGM activations, 6 orbit cameras r=1.5 fovy 49.1, "
                "seeded upstream grads); one scene per GPU",
        "config": {"workload": "cfg3: 100k Gaussians x 6 views x 256^2, render fwd+bwd (GaussianRenderer API)",
                   "gaussians": N_GAUSS, "views": VIEWS, "H": RES, "W": RES, "scenes_per_gpu": 1,
                   "pairs_K_reference": K, "pairs_binned": K_binned, "parallelism": f"scene-sharded x{world}"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": PEAK_HBM_GBS,
                     "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4), "bytes_per_launch": kb.get(dom, 0),
                     **pmc_traffic(dom)},
        "step_roofline": {"bytes": step_bytes, "achieved_GBs": round(step_bytes / (ms_step / 1e3) / 1e9, 2),
                          "frac": round(step_bytes / (ms_step / 1e3) / 1e9 / PEAK_HBM_GBS, 4)},
        "kernels": per_kernel,
    }
    if not args.no_attention:
        result["attention"] = attention_bench(dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(g_cpu, cv[None], cvp[None], tan, bg, d_img, d_alpha,
                                              args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    D.finalize(info)


if __name__ == "__main__":
    main()
