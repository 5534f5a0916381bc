"""Where the host time of a cfg3 step goes when it starts on an idle GPU (right after a synchronize: ~230 us of host
work against ~77 us in steady state, scripts/diag_first_step.py): cProfile over 20 such steps (each after 50
steady steps and a synchronize) next to 20 steady steps, top functions by total time."""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
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

    def step():
        out = r.render(g, cvd, cvpd, cpd, bg_color=bg)
        torch.autograd.backward([out["image"], out["alpha"]], [di, da])
        g.grad = None

    for _ in range(300):
        step()
    torch.cuda.synchronize()
    for name, after_sync in (("after_sync", True), ("steady", False)):
        pr = cProfile.Profile()
        for _ in range(20):
            for _ in range(50):
                step()
            if after_sync:
                torch.cuda.synchronize()
            pr.enable()
            step()
            pr.disable()
        torch.cuda.synchronize()
        buf = io.StringIO()
        pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(22)
        print(f"==== {name} (20 steps)")
        print(buf.getvalue()[-6000:])


if __name__ == "__main__":
    main()
