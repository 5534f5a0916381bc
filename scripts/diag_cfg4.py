"""Where cfg4's attention time goes (bench.py cfg4_bench's attn_pass: the 16 MVAttention blocks, bf16 autocast,
forward): the bench's host-clock time per pass, the GPU span of one pass between events, the host time to enqueue
one pass after a synchronize and in steady state, and per-kernel HIP-event times of liblgm_amd's kernels; plus a
torch profiler table of every kernel of one pass (GEMMs, casts). Usage: python scripts/diag_cfg4.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from bench import CFG4_ATTN, CFG4_FRAMES
    from lgm_amd import _native
    from lgm_amd import dist as D
    from lgm_amd.attention import MVAttention
    dev = torch.device("cuda", 0)
    torch.manual_seed(4)
    mods, xs = {}, []
    for C, S in CFG4_ATTN:
        if C not in mods:
            mods[C] = MVAttention(C, 16, num_frames=CFG4_FRAMES, skip_scale=0.5 ** 0.5).to(dev).eval()
        xs.append((mods[C], torch.randn(CFG4_FRAMES, C, S, S, device=dev)))

    def attn_pass():
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            for m, x in xs:
                m(x)

    D.warm_up(attn_pass, 2, torch.cuda.synchronize)
    steps = 20
    t0 = time.perf_counter()
    for _ in range(steps):
        attn_pass()
    torch.cuda.synchronize()
    host_clock_ms = 1e3 * (time.perf_counter() - t0) / steps
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    enq = []
    ev[0].record()
    for i in range(steps):
        h = time.perf_counter()
        attn_pass()
        enq.append(1e3 * (time.perf_counter() - h))
        ev[i + 1].record()
    torch.cuda.synchronize()
    spans = [ev[i].elapsed_time(ev[i + 1]) for i in range(steps)]
    prof = _native.KernelProfiler()
    with prof:
        for _ in range(steps):
            attn_pass()
        torch.cuda.synchronize()
    ks = {k: (n / steps, 1e3 * v / steps) for k, (n, v) in prof.summary().items()}
    prof.close()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CUDA]) as p:
        for _ in range(5):
            attn_pass()
        torch.cuda.synchronize()
    table = p.key_averages().table(sort_by="cuda_time_total", row_limit=25)
    print(json.dumps({"host_clock_ms_per_pass": round(host_clock_ms, 4),
                      "gpu_span_ms_median": round(sorted(spans)[steps // 2], 4),
                      "enqueue_ms_median": round(sorted(enq)[steps // 2], 4),
                      "lgm_kernels_us_per_pass": {k: {"launches": n, "us": round(t, 1)} for k, (n, t) in ks.items()}}))
    print(table)


if __name__ == "__main__":
    main()
