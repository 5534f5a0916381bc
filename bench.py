"""bench.py -- BASELINE.json metric: Mpixels/s of forward+backward Gaussian rasterization (256^2, 100k Gaussians,
6 views; BASELINE config 3 scenes) on 1/2/4/8 MI355X.

Workload (SURVEY.md §8(d) "scaling"): a fixed pool of 8 cfg3 scenes x 6 views (48 renders of 100k Gaussians at
256^2, seed 2), sharded by scene over the G ranks (8/G scenes per GPU, rendered by ONE batched call per rank;
no data-path collective) -> strong scaling. A step = GaussianRenderer.render (core/gs.py:31-98 API, clamp
in-kernel) of the rank's scenes + autograd backward to dL/dgaussians for fixed seeded upstream gradients of image
and alpha (LGM's loss inputs, core/models.py:141-153). value = all pixels of the pool / max-over-ranks time.

Secondary objects on the same line:
  * "cfg3_view_sharded": ONE cfg3 scene (seed 1) whose 6 views are split over the G ranks, plus the RCCL SUM
    all-reduce of dL/dgaussians [1,N,14]; at G = 1 this is exactly BASELINE config 3;
  * "cfg2": 50k Gaussians x 1 view x 256^2 forward only (BASELINE config 2), rank 0;
  * "attention": LGM's heaviest MVAttention level, bf16 fwd+bwd, MFMA and exp rooflines;
  * "cfg4": the attention blocks and the 20-view 512^2 render of one LGM 'big' forward (BASELINE config 4);
  * "cfg5": the render side of one training step (head + 26-view 512^2 render + fused loss, fwd+bwd) and the DDP
    gradient all-reduce of the UNet's 1.66 GB (BASELINE config 5);
  * "roofline": the dominant kernel priced with SURVEY §8(d)'s algorithmic bytes over its HIP-event time;
  * "cpu_baseline": the CPU oracle port on all host cores (rank 0, N = 1).

    python bench.py [--gpus N --steps K --warmup W]
With --gpus N > 1 and no torchrun environment, bench.py spawns the N ranks itself (before any GPU call).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA peak (no sparsity)
# v_exp_f32: 8 issue cycles per 64-lane wave instruction per SIMD (MI355X_MICROARCH.md constants table):
# 256 CUs x 4 SIMDs x 8 lanes/cycle x 2.4 GHz
PEAK_EXP_PER_S = 256 * 4 * 8 * 2.4e9
N_GAUSS, VIEWS, RES, POOL_SCENES = 100_000, 6, 256, 8
POOL_SEED, CFG3_SEED, CFG2_SEED = 2, 1, 0


def kernel_bytes(N, BV, K, P, B=None):
    """SURVEY.md §8(d) algorithmic bytes per launch over BV renders of B scenes: fwd = 56N + 60K + 20P,
    bwd = 112N + 84K + 28P per view, K = upstream's num_rendered summed over the views (a build that culls more is
    still credited with K_ref). k_bin (preprocess + emit) carries 56N + 8K per view, k_sort 8K. k_preproc_bwd sums
    a scene's views before the projection chain, so it is priced per SCENE: 112N (attributes in, 14 gradients out)
    plus 32 B per (view, Gaussian) of accumulators and tile rects it reads -- the per-view 112N of §8(d) would credit
    it with bytes it never moves (frac > 1)."""
    B = BV if B is None else B
    return {
        "k_bin": 56 * N * BV + 8 * K,
        "k_sort": 8 * K,
        "k_render_fwd": 44 * K + 20 * P * BV,
        "k_render_bwd": 84 * K + 28 * P * BV,
        "k_preproc_bwd": 112 * N * B + 32 * N * BV,
    }


N_SIMD, CLK_HZ = 256 * 4, 2.4e9  # MI355X: 256 CUs x 4 SIMDs; peak engine clock


def limiter_from_counters(rec, achieved_counter_gbs, avg_s=None):
    """What bounds a kernel, read off its PMC record (profiles/pmc_latest.json): HBM if the counted traffic runs at
    >= 60 % of peak; VALU issue if its VALU instructions fill >= 70 % of the chip's SIMD issue cycles over the
    launch at 2 cycles per wave64 instruction (a lower bound: MI355X_MICROARCH prices one wave's stream at 4, but
    across co-resident waves the SIMDs sustain more -- k_render_fwd's counted VALU at 4 cycles would need a 2.8 GHz
    clock -- so the 4-cycle figure, reported beside it, is an upper bound); else latency / issue (the waves wait:
    barriers, LDS and memory round trips)."""
    if not rec:
        return None
    hbm = achieved_counter_gbs / PEAK_HBM_GBS if achieved_counter_gbs else 0.0
    valu, wait = rec.get("valu_busy_frac", 0.0), rec.get("wait_frac", 0.0)
    lds = rec.get("lds_bank_conflict_frac")
    issue = None
    if avg_s and rec.get("SQ_INSTS_VALU"):
        issue = round(2.0 * rec["SQ_INSTS_VALU"] / (N_SIMD * avg_s * CLK_HZ), 4)
    kind = "hbm" if hbm >= 0.6 else "valu-issue" if (issue or 0.0) >= 0.7 else "latency/issue"
    return {"kind": kind, "hbm_frac_at_counter_bytes": round(hbm, 4), "valu_issue_frac": issue,
            "valu_issue_frac_at_4_cycles": round(2 * issue, 4) if issue is not None else None,
            "valu_busy_frac_per_wave": valu, "wait_frac": wait, "lds_bank_conflict_frac": lds}


def pmc_record(kernel):
    """HBM bytes per launch of `kernel` and its limiter counters from the committed PMC profile of this workload
    (rocprofv3 passes, gfx950-corrected: scripts/gpu_run.sh prof -> scripts/pmc_summary.py --json), or nulls."""
    path = os.path.join(ROOT, "profiles", "pmc_latest.json")
    try:
        d = json.load(open(path))
        rec = d[kernel]
        out = {"traffic": int(rec["hbm_read_bytes"] + rec["hbm_write_bytes"]),
               "traffic_source": f"profiles/pmc_latest.json ({d['_meta'].get('workload', '?')}, "
                                 f"commit {d['_meta'].get('commit', '?')})"}
        out["counters"] = {k: rec[k] for k in ("wait_frac", "valu_busy_frac", "lds_bank_conflict_frac") if k in rec}
        return out
    except (OSError, KeyError, ValueError, TypeError):
        return {"traffic": None}


def json_pmc(kernel):
    try:
        return json.load(open(os.path.join(ROOT, "profiles", "pmc_latest.json")))[kernel]
    except (OSError, KeyError, ValueError, TypeError):
        return None


def host_cpu():
    model = "?"
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    share = min(usable, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else usable
    return model, os.cpu_count() or 1, share


def cpu_baseline(g, cv, cvp, tan, bg, d_img, d_alpha, seconds):
    """The oracle port (oracle/raster_oracle.c) fwd+bwd of the cfg3 scene on the host's CPU share: OpenMP over the
    6 views x threads over each view's tiles (nested), a bounded number of repetitions."""
    from oracle import oracle as O
    O.build()
    model, ncpu, share = host_cpu()
    # nested OpenMP: `views` threads over the views x `tiles` threads over each view's tiles, every core of the share
    # busy (6 x 3 = 18 threads on a 16-core share: the per-view binning and sort run on the view's thread alone, so
    # the tile threads idle through them; fewer view threads leave cores idle there: 2 x 8 -> 0.23 Mpix/s, profiles/r02)
    views = min(VIEWS, share)
    tiles = max(1, -(-share // views))
    args = (g.numpy(), cv.numpy(), cvp.numpy(), tan, RES, RES, bg.numpy())
    kw = dict(d_image=d_img.numpy(), d_alpha=d_alpha.numpy(), nthreads=views, tile_threads=tiles)
    O.render(*args, **kw)  # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        O.render(*args, **kw)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": round(reps * VIEWS * RES * RES / el / 1e6, 3), "unit": "Mpixels/s", "cores": min(views * tiles,
                                                                                                      share),
            "threads": views * tiles, "kind": "port", "host_cpu": model, "host_cpus_visible": ncpu,
            "host_cpu_share": share,
            "sample": f"oracle/raster_oracle.c fwd+bwd of the cfg3 scene (seed 1: 100k Gaussians x 6 views x 256^2),"
                      f" {reps} repetitions in {el:.1f} s, {views} threads over views x {tiles} over tiles"}


def cpu_baseline_torch(g, cv, cvp, tan, bg, d_img, d_alpha):
    """The product's own CPU path (lgm_amd/cpu.py: vectorised torch, autograd backward; what BASELINE config 1 runs)
    on the same cfg3 scene, on every core of the share: fwd+bwd of ONE of its views (a bounded sample: the autograd
    tape of one view already holds ~6 GB)."""
    import torch

    from lgm_amd.cpu import render_cpu
    _, _, share = host_cpu()
    prev = torch.get_num_threads()
    torch.set_num_threads(share)
    try:
        gg = g.clone().requires_grad_(True)
        t0 = time.perf_counter()
        img, _, alp = render_cpu(gg, cv[:, :1], cvp[:, :1], bg, tan, tan, RES, RES, clamp=True)
        torch.autograd.backward([img, alp], [d_img[:, :1], d_alpha[:, :1]])
        el = time.perf_counter() - t0
    finally:
        torch.set_num_threads(prev)
    return {"value": round(RES * RES / el / 1e6, 4), "unit": "Mpixels/s", "cores": share, "kind": "port",
            "sample": f"lgm_amd/cpu.py render_cpu fwd+bwd (torch autograd) of view 0 of the cfg3 scene: {el:.1f} s"}


def cpu_baseline_attention(seconds):
    """the attention's CPU restatement (lgm_amd/cpu.py attention_cpu = the reference's fallback
    Attention math, core/attention.py:51-64) at LGM's heaviest level for ONE object (L = 4096, 16 heads, D = 32,
    fp32, fwd+bwd), on every core of the share; repetitions bounded by `seconds`."""
    import torch

    from lgm_amd.cpu import attention_cpu
    _, _, share = host_cpu()
    prev = torch.get_num_threads()
    torch.set_num_threads(share)
    try:
        L, H, D = 4096, 16, 32
        qkv = torch.randn(1, L, 3, H, D, generator=torch.Generator().manual_seed(7)).requires_grad_(True)
        d_o = torch.randn(1, L, H, D, generator=torch.Generator().manual_seed(8))
        reps, t0 = 0, time.perf_counter()
        while True:
            qkv.grad = None
            attention_cpu(qkv, D ** -0.5).backward(d_o)
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    finally:
        torch.set_num_threads(prev)
    flops = 14.0 * H * L * L * D * reps
    return {"value": round(flops / el / 1e12, 4), "unit": "TFLOP/s", "cores": share, "kind": "port",
            "ms_per_block": round(1e3 * el / reps, 1),
            "sample": f"attention_cpu fwd+bwd, L=4096 H=16 D=32 fp32, 1 object: {reps} repetitions in {el:.1f} s"}


def step_spread(step, n: int) -> dict:
    """Per-step GPU time of n more steps (an untimed pass, after the timed loop): CUDA events between consecutive
    steps on the current stream, min / median / max in ms -- so noise of the size of a kernel-level win is visible
    in the line next to the timed mean."""
    import torch
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    torch.cuda.synchronize()
    evs[0].record()
    for i in range(n):
        step()
        evs[i + 1].record()
    torch.cuda.synchronize()
    d = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(n))
    return {"steps": n, "min_ms": round(d[0], 4), "median_ms": round(d[n // 2], 4), "max_ms": round(d[-1], 4)}


def kernel_sum_ms(kern: dict, steps: int) -> float:
    """The profiled pass's kernel time per step (HIP events around every liblgm_amd launch), for comparison with the
    timed loop's ms_per_step: the difference is launch gaps, host stalls and non-library work (torch ops)."""
    return round(sum(ms for _, ms in kern.values()) / max(1, steps), 4)


def attention_bench(dev, steps: int = 10):
    """LGM's heaviest MVAttention level (core/unet.py:35-49 at C=512, 32x32, 4 views -> L = 4096 tokens, 16 heads,
    D = 32; 8 objects per GPU as in the 'big' training batch), bf16 fwd+bwd through the HIP kernels, torch SDPA on
    the same tensors as a comparator. FLOPs 14 B H L^2 D; exps 3 B H L^2 (forward + the two backward kernels each
    recompute P from the LSE)."""
    import torch
    import torch.nn.functional as F

    from lgm_amd import _native
    from lgm_amd import dist as Dist
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
        Dist.warm_up(fn, 1, torch.cuda.synchronize)
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
    exps = 3.0 * B * H * L * L
    tf = flops / ms / 1e9
    return {"workload": "MVAttention C=512 32x32 x 4 views (L=4096, 16 heads, D=32), 8 objects, fwd+bwd",
            "dtype": "bf16", "ms_per_step": round(ms, 4), "tflops": round(tf, 1),
            "roofline": {"bound": "mfma", "achieved": round(tf, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(tf / PEAK_BF16_TFLOPS, 4)},
            "exp_roofline": {"achieved_Gexp_s": round(exps / ms / 1e6, 1), "peak_Gexp_s": PEAK_EXP_PER_S / 1e9,
                             "frac": round(exps / (ms / 1e3) / PEAK_EXP_PER_S, 4),
                             "note": "at D=32 one exp per 128 MFMA FLOP: the v_exp_f32 issue rate bounds the "
                                     "softmax as tightly as the MFMA peak bounds the contractions"},
            "kernels": {k: {"avg_us": round(1e3 * v / n, 2), "launches": n} for k, (n, v) in kern.items()},
            "torch_sdpa_tflops": round(flops / ms_sdpa / 1e9, 1) if ms_sdpa else None}


def mva_level_bench(dev, steps: int = 10):
    """One whole MVAttention block of the bench level (core/unet.py:11-49: GroupNorm, token permute, qkv Linear,
    attention, proj Linear, permute back, residual, skip_scale; C = 512, 32x32 x 4 views, 16 heads, 8 objects),
    fwd+bwd under bf16 autocast as LGM trains: the fused HIP layout passes (lgm_mva_*, forward and backward) against
    the same module on upstream's torch ops around the same HIP attention core (fused=False). Per-kernel times of
    the fused step from a separate pass."""
    import torch

    from lgm_amd import _native
    from lgm_amd import dist as Dist
    from lgm_amd.attention import MVAttention
    B, F, C, HH, WW = 8, 4, 512, 32, 32
    torch.manual_seed(3)
    m = MVAttention(C, 16, num_frames=F, skip_scale=0.5 ** 0.5).to(dev)
    x = (torch.randn(B * F, C, HH, WW, device=dev) * 2 + 0.3).requires_grad_(True)
    gy = torch.randn(B * F, C, HH, WW, device=dev)

    def step():
        x.grad = None
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(x)
        y.backward(gy)

    def timed():
        Dist.warm_up(step, 1, torch.cuda.synchronize)
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(steps):
            step()
        en.record()
        torch.cuda.synchronize()
        return st.elapsed_time(en) / steps

    res = {"workload": f"MVAttention block C={C} {HH}x{WW} x {F} views, 16 heads, {B} objects, fwd+bwd, bf16 autocast "
                       "(GroupNorm + layout + qkv/proj Linear + attention + residual)"}
    for fused in (True, False):
        m.fused = fused
        res["fused_ms" if fused else "torch_layout_ms"] = round(timed(), 4)
    m.fused = True
    prof = _native.KernelProfiler()
    with prof:
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
    res["kernels"] = {k: {"avg_us": round(1e3 * v / n, 2), "launches": n} for k, (n, v) in prof.summary().items()
                      if k.startswith("k_mva") or k.startswith("k_wgrad")}
    prof.close()
    return res


def cfg2_bench(dev, steps):
    """BASELINE config 2: 50k Gaussians, 1 camera, 256^2, RGB+alpha forward only (bg = ones, seed 0)."""
    import torch

    from lgm_amd import GaussianRenderer, Options
    from lgm_amd.cameras import orbit_cameras
    from lgm_amd.synthetic import synthetic_gaussians
    r = GaussianRenderer(Options(output_size=RES))
    g = synthetic_gaussians(1, 50_000, seed=CFG2_SEED).to(dev)
    cv, cvp, cp = (t[None].to(dev) for t in orbit_cameras(1))
    bg = torch.ones(3, device=dev)
    from lgm_amd import _native
    from lgm_amd import dist as D
    with torch.no_grad():
        D.warm_up(lambda: r.render(g, cv, cvp, cp, bg_color=bg), 5, torch.cuda.synchronize)
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        st.record()
        for _ in range(steps):
            r.render(g, cv, cvp, cp, bg_color=bg)
        en.record()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        prof = _native.KernelProfiler()  # per-kernel HIP-event times (a separate, untimed pass)
        with prof:
            for _ in range(steps):
                r.render(g, cv, cvp, cp, bg_color=bg)
            torch.cuda.synchronize()
        kern = prof.summary()
        prof.close()
    return {"workload": "cfg2: 50k Gaussians x 1 view x 256^2, forward only", "ms_per_step": round(1e3 * el / steps, 4),
            "Mpixels_per_s": round(steps * RES * RES / el / 1e6, 2),
            "gpu_span_ms_per_step": round(st.elapsed_time(en) / steps, 4),  # (stream events around the loop)
            "kernels": {k: {"avg_us": round(1e3 * v / n, 2), "launches": n} for k, (n, v) in kern.items()}}


# LGM 'big' at BASELINE config 4 (core/options.py:93-103 with 6 input views at input_size 320, splat 160): the
# MVAttention calls of one UNet forward (core/unet.py:240-290; down levels 3-5 x 2 layers, mid x 1, up levels 0-2 x
# 3 layers) as (channels, spatial side) and the render of 20 views at 512^2 of N = 6 * 160^2 Gaussians.
CFG4_ATTN = [(512, 40)] * 2 + [(1024, 20)] * 2 + [(1024, 10)] * 2 + [(1024, 10)] + [(1024, 10)] * 3 + \
    [(1024, 20)] * 3 + [(512, 40)] * 3
CFG4_VIEWS, CFG4_FRAMES, CFG4_N, CFG4_RES = 20, 6, 6 * 160 * 160, 512


def cfg4_bench(dev, steps):
    """The hot-path share of BASELINE config 4 (LGM 'big' forward, inference): the 16 MVAttention blocks at their
    cfg4 shapes (GroupNorm + qkv + HIP flash attention + proj + residual, bf16 autocast, random init: there are no
    weights offline) and the GaussianRenderer forward of 20 views at 512^2. The UNet's convolutions / ResNet blocks
    are plain torch and out of scope; their time is not included."""
    import torch

    from lgm_amd import GaussianRenderer, Options
    from lgm_amd import dist as D
    from lgm_amd.attention import MVAttention
    from lgm_amd.cameras import orbit_cameras
    from lgm_amd.synthetic import synthetic_gaussians
    torch.manual_seed(4)
    mods = {}
    xs = []
    for C, S in CFG4_ATTN:
        if C not in mods:
            mods[C] = MVAttention(C, 16, num_frames=CFG4_FRAMES, skip_scale=0.5 ** 0.5).to(dev).eval()
        xs.append((mods[C], torch.randn(CFG4_FRAMES, C, S, S, device=dev)))

    def attn_pass():
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            for m, x in xs:
                m(x)

    r = GaussianRenderer(Options(output_size=CFG4_RES))
    g = synthetic_gaussians(1, CFG4_N, seed=4).to(dev)
    cv, cvp, cp = (t[None].to(dev) for t in orbit_cameras(CFG4_VIEWS))
    bg = torch.ones(3, device=dev)

    def render_pass():
        with torch.no_grad():
            r.render(g, cv, cvp, cp, bg_color=bg)

    def timed(fn):
        D.warm_up(fn, 2, torch.cuda.synchronize)
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - t0) / steps

    ms_attn, ms_render = timed(attn_pass), timed(render_pass)
    flops = sum(4.0 * (CFG4_FRAMES * S * S) ** 2 * C for C, S in CFG4_ATTN)  # QK^T + PV per call (B = 1)
    px = CFG4_VIEWS * CFG4_RES * CFG4_RES
    return {"workload": "cfg4 hot path: LGM 'big' (6 input views at 320 -> N = 153,600 Gaussians) -- 16 MVAttention "
                        "blocks (L = 9600 @ C512 x5, 2400 @ C1024 x5, 600 @ C1024 x6; bf16, forward) + render of 20 "
                        "views at 512^2 (forward); UNet convolutions excluded",
            "attention_ms": round(ms_attn, 4), "attention_core_tflops": round(flops / ms_attn / 1e9, 1),
            "render_ms": round(ms_render, 4), "render_Mpixels_per_s": round(px / ms_render / 1e3, 1),
            "ms_total": round(ms_attn + ms_render, 4)}


CFG5_VIEWS, CFG5_PARAMS = 26, 415_000_000  # rendered views per object; the 'big' UNet's parameter count


def cfg5_inputs(dev):
    """BASELINE config 5's render-side inputs (seeded; shared with tests/test_training_gpu.py): the Gaussian head with
    its conv set so that its Gaussians follow SURVEY §8(d)'s synthetic distribution (positions 0.35 x, scales
    0.1 softplus(x - 2.2522): median 0.01) rather than a random-init conv's metre-scale splats, a synthetic UNet
    output x [6, 14, 160, 160] (6 input views at splat 160 -> N = 153,600), 26 orbit cameras at -10 degrees, ground
    truth images / masks at 512^2 and the random training background (core/models.py:135-138)."""
    import torch

    from lgm_amd import GaussianRenderer, Options
    from lgm_amd.cameras import orbit_cameras
    from lgm_amd.head import GaussianHead
    gen = torch.Generator().manual_seed(5)
    head = GaussianHead().to(dev)
    with torch.no_grad():
        head.conv.weight.copy_(torch.diag(torch.tensor([0.35] * 3 + [1.0] * 11)).view(14, 14, 1, 1))
        head.conv.bias.zero_()
        head.conv.bias[4:7] = -2.2522
    x = torch.randn(6, 14, 160, 160, generator=gen).to(dev).requires_grad_(True)
    cv, cvp, cp = (t[None].to(dev) for t in orbit_cameras(CFG5_VIEWS, elevation=-10.0))
    gt = torch.rand(1, CFG5_VIEWS, 3, 512, 512, generator=gen).to(dev)
    mask = (torch.rand(1, CFG5_VIEWS, 1, 512, 512, generator=gen) > 0.5).float().to(dev)
    bg = torch.rand(3, generator=gen).to(dev)
    return dict(head=head, x=x, cam_view=cv, cam_view_proj=cvp, cam_pos=cp, gt=gt, mask=mask, bg=bg,
                renderer=GaussianRenderer(Options(output_size=512)))


def cfg5_bench(dev, info, steps):
    """The render side of BASELINE config 5 (main.py:82-109 training step, one object per GPU): the fused Gaussian
    head (core/models.py:96-117) on a synthetic UNet output of 6 input views at splat 160 (N = 153,600), the render of
    26 views at 512^2 with the training loss fused in (core/models.py:138-148), and the backward through both; then
    the DDP gradient exchange of the UNet's 1.66 GB fp32 gradients (100 MB buckets, fp32 on the wire as the
    reference's DDP: lgm_amd.dist.allreduce_bucketed) -- timed on its own, since the UNet itself is out of scope."""
    import torch

    from lgm_amd import dist as D
    z = cfg5_inputs(dev)
    head, x, cv, cvp, cp, gt, mask, bg, r = (z[k] for k in ("head", "x", "cam_view", "cam_view_proj", "cam_pos", "gt",
                                                            "mask", "bg", "renderer"))

    def step():
        g = head(x, 1, 6)
        out = r.render(g, cv, cvp, cp, bg_color=bg, gt_images=gt, gt_masks=mask)
        out["loss_mse"].backward()
        x.grad = None
        head.zero_grad()

    def timed(fn, n):
        D.warm_up(fn, 2, torch.cuda.synchronize, info, dev)
        return 1e3 * D.timed_steps(fn, n, info, torch.cuda.synchronize, dev) / n

    res = {"workload": "cfg5 render side (main.py:82-109, one object per GPU): Gaussian head (6 x 160^2 -> "
                       "153,600 Gaussians) + 26 views at 512^2 with the fused MSE loss, fwd+bwd; plus the DDP "
                       "all-reduce of the UNet's 1.66 GB fp32 gradients (100 MB buckets, fp32 on the wire)",
           "render_side_ms": round(timed(step, steps), 4)}
    from lgm_amd import _native
    prof = _native.KernelProfiler()  # per-kernel HIP-event times of the same step (a separate, untimed pass)
    with prof:
        for _ in range(2):
            step()
        torch.cuda.synchronize()
    res["kernels"] = {k: {"avg_us": round(1e3 * v / n, 2), "launches": n} for k, (n, v) in prof.summary().items()}
    prof.close()
    if info.world > 1:
        flat = torch.zeros(CFG5_PARAMS, device=dev)
        res["grad_allreduce_ms"] = round(timed(lambda: D.allreduce_bucketed(flat, 25_000_000, info), 3), 3)
        del flat
    else:
        res["grad_allreduce_ms"] = None
    return res


def run(args):
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

    if args.only_attn:  # the attention-side lines alone (A/B runs of the attention / MVAttention kernels)
        if rank == 0:
            print(json.dumps({"attention": attention_bench(dev), "mva_level": mva_level_bench(dev),
                              "cfg4": cfg4_bench(dev, max(10, args.steps // 5))}), flush=True)
        D.finalize(info)
        return
    renderer = GaussianRenderer(Options(output_size=RES))
    tan = float(renderer.tan_half_fov)
    cv, cvp, cp = orbit_cameras(VIEWS)

    # ---- the scaling pool: scenes s0..s1 of 8 on this rank, one batched render
    s0, s1 = D.shard_range(POOL_SCENES, rank, world)
    B = s1 - s0
    pool = synthetic_gaussians(POOL_SCENES, N_GAUSS, seed=POOL_SEED)
    d_img, _, d_alpha, bg = synthetic_upstream_grads(POOL_SCENES, VIEWS, RES, RES, seed=POOL_SEED + 1000)
    g = pool[s0:s1].contiguous().to(dev).requires_grad_(True)
    cvd = cv[None].expand(B, -1, -1, -1).contiguous().to(dev)
    cvpd = cvp[None].expand(B, -1, -1, -1).contiguous().to(dev)
    cpd = cp[None].expand(B, -1, -1).contiguous().to(dev)
    bgd = bg.to(dev)
    d_imgd, d_alphad = d_img[s0:s1].contiguous().to(dev), d_alpha[s0:s1].contiguous().to(dev)
    K_binned, K = count_pairs(g.detach(), cvd, cvpd, tan, tan, RES, RES) if B else (0, 0)

    def step():
        if B == 0:
            return
        out = renderer.render(g, cvd, cvpd, cpd, bg_color=bgd)
        torch.autograd.backward([out["image"], out["alpha"]], [d_imgd, d_alphad])
        g.grad = None

    D.warm_up(step, args.warmup, torch.cuda.synchronize, info, dev)  # (>= 50 ms: the clocks' ramp, dist.warm_up)
    # timed steps with nothing attached; per-kernel HIP-event times from a second, untimed pass of the same steps
    stamps = {}
    el = D.timed_steps(step, args.steps, info, torch.cuda.synchronize, dev, stamps=stamps)
    prof = _native.KernelProfiler()
    with prof:
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
    kern = prof.summary()
    prof.close()
    spread = step_spread(step, args.steps)

    # the same steps with bit-reproducible gradients (LGM_RENDER_DETERMINISTIC: int64 fixed-point accumulation,
    # SURVEY §5.2), timed the same way: what making it the default would cost
    det = None
    if not args.no_det and not args.only_pool:  # (PMC runs: only the headline kernels, float atomics)
        os.environ["LGM_AMD_DETERMINISTIC"] = "1"
        try:
            D.warm_up(step, max(2, args.warmup // 2), torch.cuda.synchronize, info, dev)
            n_det = max(5, args.steps // 2)
            el_det = D.timed_steps(step, n_det, info, torch.cuda.synchronize, dev)
            prof_d = _native.KernelProfiler()
            with prof_d:
                for _ in range(3):
                    step()
                torch.cuda.synchronize()
            kern_d = prof_d.summary()
            prof_d.close()
        finally:
            os.environ["LGM_AMD_DETERMINISTIC"] = "0"
        det = {"ms_per_step": round(1e3 * el_det / n_det, 4),
               "Mpixels_per_s": round(POOL_SCENES * VIEWS * RES * RES * n_det / el_det / 1e6, 2), "steps": n_det,
               "kernels": {k: {"avg_us": round(1e3 * v / n, 2), "launches": n} for k, (n, v) in kern_d.items()}}

    P = RES * RES
    pixels = POOL_SCENES * VIEWS * P * args.steps
    value = pixels / el / 1e6
    kb = kernel_bytes(N_GAUSS, B * VIEWS, K, P, B)
    per_kernel = {k: {"avg_us": round(1e3 * ms / n, 2), "launches": n} for k, (n, ms) in kern.items()}
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
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (SURVEY.md 8(d): raw~N(0,1) through LGM activations, 6 orbit cameras r=1.5 fovy 49.1, "
                "seeded upstream grads of image and alpha); scaling pool seed 2",
        "config": {"workload": f"scaling pool: {POOL_SCENES} cfg3 scenes (100k Gaussians x 6 views x 256^2 each), "
                               f"render fwd+bwd (GaussianRenderer API), sharded by scene: {B} scene(s) on rank 0",
                   "gaussians": N_GAUSS, "views": VIEWS, "H": RES, "W": RES, "pool_scenes": POOL_SCENES,
                   "scenes_per_gpu": B, "global_batch": POOL_SCENES, "pairs_K_reference_rank0": K,
                   "pairs_binned_rank0": K_binned, "parallelism": f"scene-sharded x{world} (no collective)"},
        "kernels": per_kernel,
        "step_spread": spread,
        "timed_loop": stamps,
        "profiled_kernel_sum_ms_per_step": kernel_sum_ms(kern, args.steps),
    }
    if det:
        det["slowdown_vs_float_atomics"] = round(det["ms_per_step"] / (1e3 * el / args.steps), 3)
        result["deterministic"] = det
    if kern:
        dom = max(kern.items(), key=lambda kv: kv[1][1])[0]
        dom_avg_s = kern[dom][1] / kern[dom][0] / 1e3
        achieved = kb.get(dom, 0) / dom_avg_s / 1e9
        binned = kernel_bytes(N_GAUSS, B * VIEWS, K_binned, P, B).get(dom, 0) / dom_avg_s / 1e9
        step_bytes = sum(kb.values())
        pmc = pmc_record(dom)
        counter_gbs = pmc["traffic"] / dom_avg_s / 1e9 if pmc.get("traffic") else None
        # "bound" names the roofline the kernel is priced against (the render has no contraction: HBM, SURVEY
        # §8(d)); what actually limits it is read off the counters ("limiter")
        result["roofline"] = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": PEAK_HBM_GBS,
                              "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4),
                              "bytes_per_launch": kb.get(dom, 0),
                              "frac_at_binned_K": round(binned / PEAK_HBM_GBS, 4),
                              "frac_at_counter_bytes": round(counter_gbs / PEAK_HBM_GBS, 4) if counter_gbs else None,
                              "limiter": limiter_from_counters(json_pmc(dom), counter_gbs, dom_avg_s),
                              **pmc}
        result["kernel_rooflines"] = {
            k: {"avg_us": round(1e3 * ms / n, 2), "bytes": kb.get(k), "frac": round(kb[k] / (ms / n / 1e3) / 1e9 /
                                                                                  PEAK_HBM_GBS, 4)}
            for k, (n, ms) in kern.items() if k in kb}
        result["step_roofline"] = {"bytes": step_bytes, "achieved_GBs": round(step_bytes / (ms_step / 1e3) / 1e9, 2),
                                   "frac": round(step_bytes / (ms_step / 1e3) / 1e9 / PEAK_HBM_GBS, 4)}

    if args.only_pool:
        if rank == 0:
            print(json.dumps(result), flush=True)
        D.finalize(info)
        return
    # ---- cfg3 with its views split over the ranks + one RCCL all-reduce of dL/dgaussians
    v0, v1 = D.shard_range(VIEWS, rank, world)
    g3 = synthetic_gaussians(1, N_GAUSS, seed=CFG3_SEED).to(dev).requires_grad_(True)
    d3_img, _, d3_alpha, bg3 = synthetic_upstream_grads(1, VIEWS, RES, RES, seed=CFG3_SEED + 1000)
    c3v, c3p, c3c = cv[None, v0:v1].contiguous().to(dev), cvp[None, v0:v1].contiguous().to(dev), cp[None, v0:v1].to(dev)
    d3i, d3a, bg3d = d3_img[:, v0:v1].contiguous().to(dev), d3_alpha[:, v0:v1].contiguous().to(dev), bg3.to(dev)
    ar = {"ms": 0.0}

    def step3():
        if v1 > v0:
            out = renderer.render(g3, c3v, c3p, c3c, bg_color=bg3d)
            torch.autograd.backward([out["image"], out["alpha"]], [d3i, d3a])
            grad = g3.grad
        else:
            grad = torch.zeros_like(g3)
        D.allreduce_scene_grads(grad, info)
        g3.grad = None

    D.warm_up(step3, args.warmup, torch.cuda.synchronize, info, dev)
    stamps3 = {}
    el3 = D.timed_steps(step3, args.steps, info, torch.cuda.synchronize, dev, stamps=stamps3)
    prof3 = _native.KernelProfiler()  # per-kernel times of the single-scene step (a separate, untimed pass)
    with prof3:
        for _ in range(args.steps):
            step3()
        torch.cuda.synchronize()
    kern3 = prof3.summary()
    prof3.close()
    spread3 = step_spread(step3, args.steps)
    if world > 1:  # the all-reduce on its own, same tensor size
        buf = torch.zeros(1, N_GAUSS, 14, device=dev)
        for _ in range(3):
            D.allreduce_scene_grads(buf, info)
        ar["ms"] = 1e3 * D.timed_steps(lambda: D.allreduce_scene_grads(buf, info), args.steps, info,
                                       torch.cuda.synchronize, dev) / args.steps
    result["cfg3_view_sharded"] = {
        "workload": "cfg3 (BASELINE config 3): ONE scene, 100k Gaussians x 6 views x 256^2, fwd+bwd; views split "
                    f"over {world} rank(s) + SUM all-reduce of dL/dgaussians [1,N,14] fp32 (RCCL)",
        "ms_per_step": round(1e3 * el3 / args.steps, 4),
        "Mpixels_per_s": round(VIEWS * P * args.steps / el3 / 1e6, 2),
        "allreduce_ms": round(ar["ms"], 4) if world > 1 else None,
        "step_spread": spread3, "timed_loop": stamps3, "profiled_kernel_sum_ms_per_step": kernel_sum_ms(kern3, args.steps),
        "kernels": {k: {"avg_us": round(1e3 * v / n, 2), "launches": n} for k, (n, v) in kern3.items()}}

    if not args.no_cfg5:  # every rank (its all-reduce is collective)
        result["cfg5"] = cfg5_bench(dev, info, max(10, args.steps // 5))
    if rank == 0:
        result["cfg2"] = cfg2_bench(dev, args.steps)
        if not args.no_cfg4:
            # (>= 10 timed passes: with 3 (the driver's --steps 20) one slow pass moved the mean by ~12 %:
            # cfg4 attention 2.39-2.42 ms at 5 passes vs 2.70 at 3, profiles/r05/final2)
            result["cfg4"] = cfg4_bench(dev, max(10, args.steps // 5))
        if not args.no_attention:
            result["attention"] = attention_bench(dev)
            result["mva_level"] = mva_level_bench(dev)
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(g3.detach().cpu(), cv[None], cvp[None], tan, bg3, d3_img, d3_alpha,
                                                  args.cpu_seconds)
            result["cpu_baseline_torch"] = cpu_baseline_torch(g3.detach().cpu(), cv[None], cvp[None], tan, bg3,
                                                              d3_img, d3_alpha)
            result["cpu_baseline_attention"] = cpu_baseline_attention(min(5.0, args.cpu_seconds))
            if "attention" in result:
                result["attention"]["vs_cpu_restatement"] = round(
                    result["attention"]["tflops"] / max(result["cpu_baseline_attention"]["value"], 1e-9), 1)
        print(json.dumps(result), flush=True)
    D.finalize(info)


def _rank_main(argv):
    """A rank of a self-launched multi-GPU run (lgm_amd.dist.spawn_ranks set torchrun's environment)."""
    run(parse(argv))


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-attention", action="store_true", help="skip the secondary attention measurement")
    ap.add_argument("--no-cfg4", action="store_true", help="skip the cfg4 (LGM 'big') hot-path measurement")
    ap.add_argument("--no-cfg5", action="store_true", help="skip the cfg5 (training step, render side) measurement")
    ap.add_argument("--no-det", action="store_true", help="skip the deterministic-mode timing of the pool")
    ap.add_argument("--only-attn", action="store_true",
                    help="only the attention, MVAttention-level and cfg4 lines (attention-side A/B runs)")
    ap.add_argument("--only-pool", action="store_true",
                    help="only the headline workload (for counter profiles: no other kernel launches of other sizes)")
    return ap.parse_args(argv)


def main():
    args = parse()
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if "RANK" in os.environ:
        if args.gpus != world_env:
            raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world_env} from the launcher")
        run(args)
    elif args.gpus > 1:
        # no launcher: start the ranks here, before anything touches the GPU (children, not an exec)
        from lgm_amd import dist as D
        D.spawn_ranks(_rank_main, args.gpus, sys.argv[1:])
    else:
        run(args)


if __name__ == "__main__":
    main()
