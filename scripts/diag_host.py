"""Host overhead of bench.py's single-scene (cfg3) step: per-step host time (the Python / autograd / C-ABI launch
work, no sync) next to the GPU's per-step time (events between steps), the garbage collections that ran inside
the loop, and the timed mean -- to tell whether the timed loop is host-starved.
--pool-first runs bench.py's 8-scene pool steps first (as bench.py does before its cfg3 loop) and --warmup sets
the single-scene warmup; the per-step (host, GPU) times of the first 12 timed steps are printed too.
--idle-ms sleeps (GPU idle) before the loop; gpu_us_by_20 = mean GPU time per step over each 20 steps.
Usage: python scripts/diag_host.py [--steps 200] [--warmup 20] [--gc off|on|freeze|collect] [--pool-first]
       [--idle-ms MS]"""
import argparse
import gc
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--gc", default="on", choices=["on", "off", "freeze", "collect"])
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--pool-first", action="store_true")
    ap.add_argument("--idle-ms", type=float, default=0.0, help="sleep this long (GPU idle) before the timed loop")
    a = ap.parse_args()
    import torch
    from bench import CFG3_SEED, N_GAUSS, POOL_SCENES, POOL_SEED, RES, VIEWS
    from lgm_amd import GaussianRenderer, Options
    from lgm_amd.cameras import orbit_cameras
    from lgm_amd.synthetic import synthetic_gaussians, synthetic_upstream_grads

    dev = torch.device("cuda", 0)
    r = GaussianRenderer(Options(output_size=RES))
    cv, cvp, cp = orbit_cameras(VIEWS)
    g3 = synthetic_gaussians(1, N_GAUSS, seed=CFG3_SEED).to(dev).requires_grad_(True)
    d3i, _, d3a, bg3 = synthetic_upstream_grads(1, VIEWS, RES, RES, seed=CFG3_SEED + 1000)
    cvd, cvpd, cpd = cv[None].contiguous().to(dev), cvp[None].contiguous().to(dev), cp[None].to(dev)
    d3i, d3a, bg3 = d3i.contiguous().to(dev), d3a.contiguous().to(dev), bg3.to(dev)

    def step():
        out = r.render(g3, cvd, cvpd, cpd, bg_color=bg3)
        torch.autograd.backward([out["image"], out["alpha"]], [d3i, d3a])
        g3.grad = None

    if a.pool_first:
        gp = synthetic_gaussians(POOL_SCENES, N_GAUSS, seed=POOL_SEED).to(dev).requires_grad_(True)
        dpi, _, dpa, bgp = synthetic_upstream_grads(POOL_SCENES, VIEWS, RES, RES, seed=POOL_SEED + 1000)
        B = POOL_SCENES
        cvb, cvpb = (x[None].expand(B, -1, -1, -1).contiguous().to(dev) for x in (cv, cvp))
        cpb = cp[None].expand(B, -1, -1).contiguous().to(dev)
        dpi, dpa, bgp = dpi.to(dev), dpa.to(dev), bgp.to(dev)
        for _ in range(40):
            out = r.render(gp, cvb, cvpb, cpb, bg_color=bgp)
            torch.autograd.backward([out["image"], out["alpha"]], [dpi, dpa])
            gp.grad = None
        del out
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    gcs = []
    t_gc = {}

    def cb(phase, info):
        if phase == "start":
            t_gc["t"] = time.perf_counter()
        else:
            gcs.append((info["generation"], 1e6 * (time.perf_counter() - t_gc["t"])))
    gc.callbacks.append(cb)
    if a.gc == "off":
        gc.disable()
    elif a.gc == "collect":
        gc.collect()
    elif a.gc == "freeze":
        gc.collect()
        gc.freeze()
    n = a.steps
    if a.idle_ms > 0:
        torch.cuda.synchronize()
        time.sleep(a.idle_ms / 1e3)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    host = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evs[0].record()
    for i in range(n):
        h0 = time.perf_counter()
        step()
        host.append(1e6 * (time.perf_counter() - h0))
        evs[i + 1].record()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    gc.callbacks.remove(cb)
    gc.enable()
    gpu = [1e3 * evs[i].elapsed_time(evs[i + 1]) for i in range(n)]

    def st(x):
        s = sorted(x)
        return {"min": round(s[0], 1), "median": round(statistics.median(s), 1), "p90": round(s[int(0.9 * len(s))], 1),
                "max": round(s[-1], 1), "mean": round(statistics.fmean(s), 1)}
    print(json.dumps({"gc": a.gc, "steps": n, "timed_mean_us": round(1e6 * el / n, 1), "host_us": st(host),
                      "gpu_us": st(gpu), "gc_runs": len(gcs),
                      "gc_us_by_gen": {gen: round(sum(t for g, t in gcs if g == gen), 1) for gen in (0, 1, 2)},
                      "idle_ms": a.idle_ms,
                      "gpu_us_by_20": [round(statistics.fmean(gpu[i:i + 20]), 1) for i in range(0, n, 20)],
                      "first12": [(round(host[i], 1), round(gpu[i], 1)) for i in range(min(12, n))],
                      "slow_steps": [(i, round(host[i], 1), round(gpu[i], 1)) for i in range(n) if gpu[i] > 260][:20]}))


if __name__ == "__main__":
    main()
