"""Per-level cost of one MVAttention block at BASELINE config 4's shapes (bf16 autocast, inference): GPU time per
call (events over back-to-back calls), host issue time of a call with an idle queue, and liblgm_amd's kernel times."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lgm_amd import _native  # noqa: E402
from lgm_amd.attention import MVAttention  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(4)
for C, S in ((512, 40), (1024, 20), (1024, 10)):
    m = MVAttention(C, 16, num_frames=6, skip_scale=0.5 ** 0.5).to(dev).eval()
    x = torch.randn(6, C, S, S, device=dev)
    res = {"C": C, "S": S}
    for fused in (True, False):
        m.fused = fused

        def call():
            with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
                m(x)

        for _ in range(3):
            call()
        torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(20):
            call()
        en.record()
        torch.cuda.synchronize()
        host = []
        for _ in range(10):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            call()
            host.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        prof = _native.KernelProfiler()
        with prof:
            for _ in range(10):
                call()
            torch.cuda.synchronize()
        k = prof.summary()
        prof.close()
        tag = "fused" if fused else "torch"
        res[tag] = {"us_per_call": round(1e3 * st.elapsed_time(en) / 20, 1),
                    "host_us": round(1e6 * sorted(host)[5], 1),
                    "kernels_us": {n: round(1e3 * ms / c, 1) for n, (c, ms) in k.items()}}
    print(json.dumps(res), flush=True)
