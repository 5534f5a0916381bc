"""Host enqueue latency of a cfg3 step that starts on an idle GPU (the first step of every timed loop: bench.py's
timed_loop stamps show it at ~0.38 ms of host time against ~0.09 ms in steady state). Each iteration: synchronize,
then time the host work of render() and of autograd's backward separately, then the GPU span of the step (events)
-- compared with a trivial torch op after a synchronize (the bare launch-after-idle cost) and with steady-state
(back-to-back) steps. Usage: python scripts/diag_first_step.py [--iters 20]"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import torch
    from bench import CFG3_SEED, N_GAUSS, RES, VIEWS
    from lgm_amd import GaussianRenderer, Options
    from lgm_amd.cameras import orbit_cameras
    from lgm_amd.synthetic import synthetic_gaussians, synthetic_upstream_grads

    dev = torch.device("cuda", 0)
    r = GaussianRenderer(Options(output_size=RES))
    cv, cvp, cp = orbit_cameras(VIEWS)
    g = synthetic_gaussians(1, N_GAUSS, seed=CFG3_SEED).to(dev).requires_grad_(True)
    di, _, da, bg = synthetic_upstream_grads(1, VIEWS, RES, RES, seed=CFG3_SEED + 1000)
    cvd, cvpd, cpd = cv[None].contiguous().to(dev), cvp[None].contiguous().to(dev), cp[None].to(dev)
    di, da, bg = di.contiguous().to(dev), da.contiguous().to(dev), bg.to(dev)
    x = torch.zeros(16, device=dev)

    def step():
        out = r.render(g, cvd, cvpd, cpd, bg_color=bg)
        torch.autograd.backward([out["image"], out["alpha"]], [di, da])
        g.grad = None

    for _ in range(300):  # warm (clocks, caches, allocator)
        step()
    torch.cuda.synchronize()
    res = {"after_sync": {"render_us": [], "backward_us": [], "gpu_us": []}, "trivial_op_us": [],
           "steady": {"host_us": [], "gpu_us": []}}
    for _ in range(a.iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        x.add_(1.0)
        res["trivial_op_us"].append(1e6 * (time.perf_counter() - t0))
        for _ in range(50):  # keep the clocks up between the samples
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        out = r.render(g, cvd, cvpd, cpd, bg_color=bg)
        t1 = time.perf_counter()
        torch.autograd.backward([out["image"], out["alpha"]], [di, da])
        g.grad = None
        t2 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        s = res["after_sync"]
        s["render_us"].append(1e6 * (t1 - t0))
        s["backward_us"].append(1e6 * (t2 - t1))
        s["gpu_us"].append(1e3 * e0.elapsed_time(e1))
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(a.iters + 1)]
    evs[0].record()
    for i in range(a.iters):
        h = time.perf_counter()
        step()
        res["steady"]["host_us"].append(1e6 * (time.perf_counter() - h))
        evs[i + 1].record()
    torch.cuda.synchronize()
    res["steady"]["gpu_us"] = [1e3 * evs[i].elapsed_time(evs[i + 1]) for i in range(a.iters)]

    def summ(v):
        return {"median": round(statistics.median(v), 1), "min": round(min(v), 1), "max": round(max(v), 1)}
    out = {"after_sync": {k: summ(v) for k, v in res["after_sync"].items()}, "trivial_op_us": summ(res["trivial_op_us"]),
           "steady": {k: summ(v) for k, v in res["steady"].items()}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
