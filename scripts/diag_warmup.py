"""Round-5 diagnosis of BENCH_r04's pool stall (timed mean 6.5 % above the same run's median step): the driver's
`bench.py --steps 20 --warmup 5` with the round-4 warm-up (whose rate estimate included the first, one-time-cost
call), printing the per-step stamps of the timed loop. Run as `python scripts/diag_warmup.py --steps 20 --warmup 5
--only-pool`; compare with bench.py's own line."""
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from lgm_amd import dist as D  # noqa: E402


def legacy_warm_up(step, steps, sync, info=None, device=None, min_seconds=0.05):
    steps = max(1, steps)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    el = time.perf_counter() - t0
    extra = math.ceil(max(0.0, min_seconds - el) / (el / steps)) if el > 0 else 0
    print(f"legacy warm-up: {steps} steps in {1e3 * el:.1f} ms -> {extra} extra", file=sys.stderr)
    for _ in range(extra):
        step()
    sync()
    return steps + extra


if __name__ == "__main__":
    D.warm_up = legacy_warm_up
    bench.run(bench.parse())
