"""GPU parity of the HIP render path (through the C ABI) against the CPU oracle (oracle/raster_oracle.c).

Tolerances (north_star, BASELINE.json: "within 1e-4 rel L2 (fp32)"):
  * forward outputs (image, depth, alpha): relative L2 < 1e-4 against the fp32 oracle;
  * gradients dL/dgaussians, per parameter group: relative L2 against the SAME algorithm evaluated in fp64
    (oracle built with -DLGM_ORACLE_F64) must not exceed max(1e-4, 1.25 x the fp32 oracle's own error against
    fp64). Rationale: a few ill-conditioned Gaussians (needles, near-clamped) make the rotation/scale gradients
    fp32-noise-limited -- at cfg3 the faithful fp32 restatement itself is 1.9e-4 (d_rot) and 1.0e-4 (d_scale)
    away from fp64, so 1e-4 between two fp32 implementations is below the algorithm's own noise floor there;
    the GPU must be as accurate as a faithful fp32 implementation. Parity of the oracle itself is UNPINNED against the real upstream CUDA code
(see oracle/raster_oracle.c header)."""
import numpy as np
import pytest
import torch

from lgm_amd import gs as lgs
from lgm_amd.gs import rasterize
from tests.render_cases import TAN, grad_bar, near_threshold_records, rel_l2, scene, upstream

pytestmark = pytest.mark.gpu

FWD_TOL = 1e-4
BWD_TOL = 1e-4
GROUPS = {"mean": slice(0, 3), "opacity": slice(3, 4), "scale": slice(4, 7), "rot": slice(7, 11), "rgb": slice(11, 14)}


def _run(cuda, g, cv, cvp, H, W, bg, mod=1.0, grads=None, no_cull=False):
    gd = g.to(cuda).requires_grad_(grads is not None)
    img, dep, alp = rasterize(gd, cv.to(cuda), cvp.to(cuda), bg.to(cuda), TAN, TAN, H, W, mod, no_cull=no_cull)
    out = {"image": img.detach().cpu().numpy(), "depth": dep.detach().cpu().numpy(),
           "alpha": alp.detach().cpu().numpy()}
    if grads is not None:
        d_img, d_dep, d_alp = grads
        loss = (img * d_img.to(cuda)).sum() + (dep * d_dep.to(cuda)).sum() + (alp * d_alp.to(cuda)).sum()
        loss.backward()
        out["d_gaussians"] = gd.grad.cpu().numpy()
    torch.cuda.synchronize()
    return out


def _oracle(O, g, cv, cvp, H, W, bg, mod=1.0, grads=None):
    kw = {}
    if grads is not None:
        kw = dict(d_image=grads[0].numpy(), d_depth=grads[1].numpy(), d_alpha=grads[2].numpy())
    out = O.render(g.numpy(), cv.numpy(), cvp.numpy(), TAN, H, W, bg.numpy(), scale_modifier=mod, **kw)
    if grads is not None:
        out["truth"] = O.render(g.numpy(), cv.numpy(), cvp.numpy(), TAN, H, W, bg.numpy(), scale_modifier=mod,
                                f64=True, **kw)["d_gaussians"]
    return out


def _check_fwd(out, ref, tol=FWD_TOL):
    for k in ("image", "depth", "alpha"):
        e = rel_l2(out[k], ref[k])
        assert e < tol, f"{k}: rel L2 {e:.3e}"


def _check_bwd(out, ref, tol=BWD_TOL):
    truth = ref["truth"]
    for name, sl in GROUPS.items():
        e_gpu = rel_l2(out["d_gaussians"][..., sl], truth[..., sl])
        e_o32 = rel_l2(ref["d_gaussians"][..., sl], truth[..., sl])
        assert e_gpu < grad_bar(e_o32, tol), f"d_{name}: GPU vs fp64 {e_gpu:.3e}, fp32 oracle vs fp64 {e_o32:.3e}"


@pytest.mark.parametrize("B,N,V,H,W,mod", [(1, 1, 1, 32, 32, 1.0), (1, 300, 2, 64, 64, 1.0), (2, 2000, 3, 64, 64, 1.0),
                                           (1, 3000, 2, 50, 50, 0.7), (1, 2500, 2, 40, 72, 1.0),
                                           (2, 1500, 2, 128, 128, 1.3),
                                           (1, 400, 34, 32, 32, 1.0)])  # > PRE_MAXV views: k_preproc_bwd<false>
def test_forward_backward_parity(cuda, oracle_mod, B, N, V, H, W, mod):
    g, cv, cvp = scene(B=B, N=N, V=V, seed=N + V)
    grads = upstream(B, V, H, W)
    bg = grads[3]
    out = _run(cuda, g, cv, cvp, H, W, bg, mod, grads[:3])
    ref = _oracle(oracle_mod, g, cv, cvp, H, W, bg, mod, grads[:3])
    _check_fwd(out, ref)
    _check_bwd(out, ref)


def test_empty_and_culled(cuda, oracle_mod):
    # N = 0: pure background; all-culled (behind the near plane): pure background, zero gradients
    bg = torch.tensor([0.1, 0.2, 0.3])
    g, cv, cvp = scene(N=64, V=2, seed=3)
    out = _run(cuda, g[:, :0].contiguous(), cv, cvp, 32, 32, bg)
    assert np.allclose(out["image"], bg.view(1, 1, 3, 1, 1).numpy().repeat(32, 3).repeat(32, 4))
    assert np.all(out["alpha"] == 0)
    g2 = g.clone()
    g2[..., 0:3] = torch.tensor([0.0, 0.0, 1.45])  # at the camera of view 0 (depth <= 0.2) ...
    g2[..., 2] = 1.45
    grads = upstream(1, 2, 32, 32)
    out = _run(cuda, g2, cv[:, :1], cvp[:, :1], 32, 32, bg, grads=tuple(x[:, :1] for x in grads[:3]))
    ref = _oracle(oracle_mod, g2, cv[:, :1], cvp[:, :1], 32, 32, bg, grads=tuple(x[:, :1] for x in grads[:3]))
    assert np.allclose(out["image"], ref["image"], atol=1e-6)
    assert np.abs(out["d_gaussians"]).max() == 0.0


def test_oversized_tile_bucket(cuda, oracle_mod):
    # > 8192 Gaussians in the centre tiles: exercises the LDS-chunk + global-merge sort path
    g, cv, cvp = scene(N=20000, V=1, seed=11, shrink=0.02, scale_mul=0.05)
    grads = upstream(1, 1, 64, 64)
    out = _run(cuda, g, cv, cvp, 64, 64, grads[3], grads=grads[:3])
    ref = _oracle(oracle_mod, g, cv, cvp, 64, 64, grads[3], grads=grads[:3])
    _check_fwd(out, ref)
    _check_bwd(out, ref)


def test_exact_count_path(cuda, oracle_mod, monkeypatch):
    # force the sync-once exact pair-count workspace path
    monkeypatch.setattr(lgs, "_WS_BUDGET", 0)
    g, cv, cvp = scene(N=3000, V=2, seed=5)
    grads = upstream(1, 2, 64, 64)
    out = _run(cuda, g, cv, cvp, 64, 64, grads[3], grads=grads[:3])
    ref = _oracle(oracle_mod, g, cv, cvp, 64, 64, grads[3], grads=grads[:3])
    _check_fwd(out, ref)
    _check_bwd(out, ref)


def test_forward_deterministic(cuda):
    g, cv, cvp = scene(N=20000, V=2, seed=2)
    bg = torch.ones(3)
    a = _run(cuda, g, cv, cvp, 128, 128, bg)
    b = _run(cuda, g, cv, cvp, 128, 128, bg)
    for k in a:
        assert np.array_equal(a[k], b[k]), k


def test_repeated_backward_retain_graph(cuda):
    """A second backward of one forward (retain_graph) gives the first one's gradient: the forward zeroes
    the accumulators, and the repeat clears what the first backward left (LGM_RENDER_BACKWARD_AGAIN)."""
    g, cv, cvp = scene(N=3000, V=2, seed=5)
    gd = g.to(cuda).requires_grad_(True)
    img, _, alp = rasterize(gd, cv.to(cuda), cvp.to(cuda), torch.ones(3, device=cuda), TAN, TAN, 64, 64)
    w = torch.randn(img.shape, generator=torch.Generator().manual_seed(3)).to(cuda)
    loss = (img * w).sum() + alp.sum()
    (first,) = torch.autograd.grad(loss, gd, retain_graph=True)
    (second,) = torch.autograd.grad(loss, gd)
    torch.cuda.synchronize()
    assert first.abs().sum().item() > 0
    # the same sums in a different atomic order: equal to fp32 rounding
    assert rel_l2(second.cpu().numpy(), first.cpu().numpy()) < 1e-5


@pytest.mark.parametrize("V", [2, 6])
def test_deterministic_saturation_poisons_and_resets(cuda, V):
    """LGM_RENDER_DETERMINISTIC's overflow guard (render_raster.hip k_render_bwd flush): a flush above its record's
    bound (2^62 / 2^ceil(log2 F), F = T flushes for a per-view record, V * T for a per-scene one:
    lgm_render_det_flush_limit_log2, tests/test_abi.py) is counted and k_preproc_bwd poisons the call's gradients
    with NaN. The lgm_diag test hook lowers the bound to 2^1 to force that path; a retain_graph repeat of the same
    forward without the hook (LGM_RENDER_BACKWARD_AGAIN) must not inherit the count (k_det_seed_max clears it), stays
    below the derived multi-view bounds (finite) and equals a clean backward bitwise."""
    from lgm_amd import _native
    g, cv, cvp = scene(N=3000, V=V, seed=5)
    gd = g.to(cuda).requires_grad_(True)
    args = (cv.to(cuda), cvp.to(cuda), torch.ones(3, device=cuda), TAN, TAN, 64, 64)
    w = torch.randn((1, V, 3, 64, 64), generator=torch.Generator().manual_seed(3)).to(cuda)
    img, _, alp = rasterize(gd, *args, deterministic=True)
    loss = (img * w).sum() + alp.sum()
    with _native.diagnostics(det_limit_log2=1):
        (poisoned,) = torch.autograd.grad(loss, gd, retain_graph=True)
    (again,) = torch.autograd.grad(loss, gd)
    img2, _, alp2 = rasterize(gd, *args, deterministic=True)
    (clean,) = torch.autograd.grad((img2 * w).sum() + alp2.sum(), gd)
    torch.cuda.synchronize()
    assert torch.isnan(poisoned).all()
    assert torch.isfinite(again).all() and again.abs().sum().item() > 0
    assert torch.equal(again, clean)


def test_cfg2_full_size_forward(cuda, oracle_mod):
    # BASELINE config 2: 50k Gaussians, 1 camera, 256^2, fwd only (seed 0)
    g, cv, cvp = scene(N=50000, V=1, seed=0)
    bg = torch.ones(3)
    out = _run(cuda, g, cv, cvp, 256, 256, bg)
    ref = _oracle(oracle_mod, g, cv, cvp, 256, 256, bg)
    _check_fwd(out, ref)


def test_cfg3_full_size_fwd_bwd(cuda, oracle_mod):
    # BASELINE config 3: 100k Gaussians, 6 views, 256^2, fwd + bwd (seed 1)
    g, cv, cvp = scene(N=100000, V=6, seed=1)
    grads = upstream(1, 6, 256, 256, seed=2)
    out = _run(cuda, g, cv, cvp, 256, 256, grads[3], grads=grads[:3])
    ref = _oracle(oracle_mod, g, cv, cvp, 256, 256, grads[3], grads=grads[:3])
    _check_fwd(out, ref)
    _check_bwd(out, ref)


def test_renderer_module_api(cuda):
    from lgm_amd import GaussianRenderer, Options
    opt = Options(output_size=64)
    r = GaussianRenderer(opt)
    g, cv, cvp = scene(B=2, N=500, V=3, seed=9)
    cp = torch.zeros(2, 3, 3)
    out = r.render(g.to(cuda).half(), cv.to(cuda), cvp.to(cuda), cp.to(cuda))
    assert out["image"].shape == (2, 3, 3, 64, 64) and out["alpha"].shape == (2, 3, 1, 64, 64)
    assert out["depth"].shape == (2, 3, 1, 64, 64)
    assert float(out["image"].min()) >= 0 and float(out["image"].max()) <= 1
    opt.output_size = 32  # convert.py mutates output_size between calls
    assert r.render(g.to(cuda), cv.to(cuda), cvp.to(cuda), cp.to(cuda))["image"].shape[-1] == 32
    # fp16 input -> fp16 gradient through the cast, as core/gs.py:45-49's .float() does
    gh = g.to(cuda).half().requires_grad_(True)
    r.render(gh, cv.to(cuda), cvp.to(cuda), cp.to(cuda))["image"].sum().backward()
    assert gh.grad is not None and gh.grad.dtype == torch.float16


@pytest.mark.parametrize("N", [600, 3000, 12000])
def test_equal_depth_ties(cuda, oracle_mod, N):
    # a flat layer (z = 0) seen head-on from the azimuth-0 orbit camera: every depth is exactly 1.5, so the tile
    # order is decided purely by Gaussian id (upstream's stable sort) -- exercises the id-digit radix passes, and
    # at N = 12000 the oversized-bucket path.
    g, cv, cvp = scene(N=N, V=1, seed=N)
    g[..., 2] = 0.0
    g[..., 0:2] *= 0.6
    grads = upstream(1, 1, 48, 48)
    out = _run(cuda, g, cv, cvp, 48, 48, grads[3], grads=grads[:3])
    ref = _oracle(oracle_mod, g, cv, cvp, 48, 48, grads[3], grads=grads[:3])
    _check_fwd(out, ref)
    _check_bwd(out, ref)


def test_exact_culling_is_output_preserving(cuda):
    """The exact opacity-aware tile culling drops only (Gaussian, tile) pairs that every pixel would skip: the
    forward is bitwise identical with and without it; gradients agree to float-atomic reordering."""
    g, cv, cvp = scene(N=30000, V=2, seed=21)
    grads = upstream(1, 2, 128, 128)
    full = _run(cuda, g, cv, cvp, 128, 128, grads[3], grads=grads[:3], no_cull=True)  # per-call LGM_RENDER_NO_CULL
    culled = _run(cuda, g, cv, cvp, 128, 128, grads[3], grads=grads[:3])
    for k in ("image", "depth", "alpha"):
        assert np.array_equal(full[k], culled[k]), k
    assert rel_l2(culled["d_gaussians"], full["d_gaussians"]) < 1e-5


def test_fused_clamp_matches_torch_clamp(cuda):
    """LGM_RENDER_CLAMP_IMAGE == core/gs.py:87's image.clamp(0, 1) and its autograd: the forward equals clamp of
    the unclamped image bitwise, the gradient equals the unclamped path fed torch's clamp mask (inclusive)."""
    g, cv, cvp = scene(B=2, N=3000, V=2, seed=33)
    g[..., 11:14] = g[..., 11:14] * 2.2 - 0.6  # colours outside [0, 1] so both clamp bounds are hit
    d_img, _, d_alp, bg = upstream(2, 2, 64, 64)
    outs = {}
    for clamp in (False, True):
        gd = g.to(cuda).requires_grad_(True)
        img, _, alp = rasterize(gd, cv.to(cuda), cvp.to(cuda), bg.to(cuda), TAN, TAN, 64, 64, clamp=clamp)
        if clamp:
            up = d_img.to(cuda)
        else:
            raw = img.detach()
            outs["raw"] = raw
            up = d_img.to(cuda) * ((raw >= 0) & (raw <= 1)).float()
        ((img * up).sum() + (alp * d_alp.to(cuda)).sum()).backward()
        outs[clamp] = (img.detach(), gd.grad.clone())
    raw = outs["raw"]
    frac = float(((raw < 0) | (raw > 1)).float().mean())
    assert 0.01 < frac < 0.9, frac  # the clamp is actually exercised
    assert torch.equal(outs[True][0], raw.clamp(0, 1))
    assert rel_l2(outs[True][1].cpu().numpy(), outs[False][1].cpu().numpy()) < 1e-5


def test_needle_decision_is_contraction_free(cuda):
    """rec_needle on the GPU (lgm_render_needle_flags: the function the binning's flag and the backward flush's
    re-derivation both call, render_bin.hip / render_raster.hip) decides every near-threshold record exactly as the
    separately rounded IEEE expression, including those where an FMA contraction would flip it."""
    from lgm_amd import _native
    recs, dec = near_threshold_records()
    abc = torch.from_numpy(recs).to(cuda)
    flags = torch.empty(len(recs), dtype=torch.uint8, device=cuda)
    _native.check(_native.lib().lgm_render_needle_flags(len(recs), _native.ptr(abc), _native.ptr(flags),
                                                        _native.stream_of(cuda)), "lgm_render_needle_flags")
    got = flags.cpu().numpy().astype(bool)
    assert np.array_equal(got, dec[:, 0]), f"{int((got != dec[:, 0]).sum())} decisions differ"
    assert (got != dec[:, 1]).any() or (got != dec[:, 2]).any()


def test_needle_flag_is_a_function_of_the_stored_record(cuda):
    """Float mode sends a needle-like record's conic partials to fp64 side accumulators; the binning flags the record
    (bit 31 of its rect, read by the preprocess backward) from the record in registers, the backward's flush
    re-derives the flag from the record loaded back from memory (render_common.h rec_needle). They agree only if
    the decision is a pure function of the stored bits: FP contraction off, separately rounded IEEE operations.
    Checked on every visible record of cfg4's 512^2 needle-heavy scene (5 views): the binning's flag equals the
    same expression evaluated in float32 by numpy on the stored (A', B', C'), including the records nearest the
    threshold (condition 300)."""
    from lgm_amd.gs import forward_state
    from lgm_amd.synthetic import synthetic_gaussians
    from lgm_amd.cameras import orbit_cameras
    g = synthetic_gaussians(1, 153_600, seed=4)
    cv, cvp, _ = orbit_cameras(20)
    cv, cvp = cv[None, 0:20:4].contiguous(), cvp[None, 0:20:4].contiguous()
    st = forward_state(g.to(cuda), cv.to(cuda), cvp.to(cuda), TAN, TAN, 512, 512, records=True)
    P, Q, rects = st["P"].reshape(-1, 4), st["Q"].reshape(-1, 4), st["rects"].reshape(-1, 2)
    vis = (rects[:, 0] & 0xFFFF) != (rects[:, 1] & 0xFFFF)
    Ap, Bp, Cp = P[vis, 2], P[vis, 3], Q[vis, 0]
    f32 = np.float32
    sac = (Ap + Cp).astype(f32)
    dq = (Ap * Cp).astype(f32) - ((f32(0.25) * Bp).astype(f32) * Bp).astype(f32)
    with np.errstate(invalid="ignore", over="ignore"):
        needle = ~((sac * sac).astype(f32) <= (f32(300.0) * dq).astype(f32))
        flag = (rects[vis, 1] >> 31).astype(bool)
        cond = (sac.astype(np.float64) ** 2) / dq.astype(np.float64)
    near = np.sort(np.abs(cond[np.isfinite(cond) & (dq > 0)] / 300.0 - 1.0))[:5]
    print(f"{int(vis.sum())} visible records, {int(needle.sum())} needles; nearest |cond/300 - 1|: {near}")
    assert needle.sum() > 0
    assert np.array_equal(flag, needle), f"{int((flag != needle).sum())} records flagged differently"
