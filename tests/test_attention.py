"""Multi-view attention: oracle pinned to the reference's own modules (tests/golden/attn_*.npz, made by
tests/golden/make_attn_golden.py from core/attention.py + core/unet.py), and the HIP flash-attention path
(lgm_amd/attention.py -> lgm_attn_* in liblgm_amd.so) checked against them on the GPU.

Tolerances: fp32 inputs -> 1e-4 relative L2 against the reference (the north_star bar; the exact-f32 MFMA path
lands around 1e-6). bf16 / fp16 compute is compared with the fp64 result of the same rounded inputs:
bf16 2e-2, fp16 3e-3 relative L2 (P and dS are rounded to the 8-/11-bit mantissa before the second MFMA).
"""
import ast
import glob
import os

import numpy as np
import pytest
import torch

from oracle import attention_ref as ref
from render_cases import rel_l2

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "attn_*.npz")))


class _Seeded:
    """Expected values of a seeded fixture (LGM's real widths, make_attn_golden.py): a strided sample of each output
    plus its full float64 L2 norm; `close` compares a computed array on both."""

    def __init__(self, z, key):
        self.idx, self.val = z["idx." + key], z["sample." + key]
        self.norm = float(z["norm." + key])

    def err(self, a):
        a = np.asarray(a, np.float64).reshape(-1)
        return max(rel_l2(a[self.idx], self.val), abs(float(np.linalg.norm(a)) - self.norm) / max(self.norm, 1e-30))


def _load(path):
    """(meta, z, params, grads): z["x"], z["gy"] the inputs, z["y"], z["dx"] and grads[name] the reference's outputs
    -- arrays, or _Seeded samples for the seeded fixtures, whose inputs are regenerated here exactly as
    make_attn_golden.py drew them."""
    z = np.load(path)  # allow_pickle=False (default): plain arrays only
    meta = ast.literal_eval(str(z["meta"]))
    if meta.get("seeded"):
        from tests.golden.make_attn_golden import seeded_inputs
        name = os.path.basename(path)[5:-4]
        params, x, draw_gy = seeded_inputs(name, meta["params"], meta["shape"])
        zz = {"x": x.numpy(), "gy": draw_gy(tuple(meta["shape"])).numpy(), "y": _Seeded(z, "y"), "dx": _Seeded(z, "dx")}
        grads = {k: _Seeded(z, "grad." + k) for k, _ in meta["params"]}
        return meta, zz, params, grads
    params = {k[6:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("param.")}
    grads = {k[5:]: z[k] for k in z.files if k.startswith("grad.")}
    return meta, z, params, grads


def _err(got, want):
    """rel L2 of a computed array against a fixture array or a _Seeded sample."""
    return want.err(got) if isinstance(want, _Seeded) else rel_l2(got, want)


def _oracle_fn(meta, params):
    if meta["kind"] == "memeff":
        return lambda x, p: ref.attention(x, p, meta["num_heads"])
    return lambda x, p: ref.mv_attention(x, p, meta["num_heads"], meta["num_frames"], meta["skip_scale"])


def _module(meta):
    from lgm_amd.attention import MemEffAttention, MVAttention
    if meta["kind"] == "memeff":
        return MemEffAttention(meta["dim"], meta["num_heads"], qkv_bias=False, proj_bias=True)
    return MVAttention(meta["dim"], meta["num_heads"], num_frames=meta["num_frames"], skip_scale=meta["skip_scale"])


def test_golden_present():
    assert len(GOLDEN) >= 13
    names = [os.path.basename(p) for p in GOLDEN]
    # LGM's real channel widths with 16 heads (core/unet.py:113-206): D = 32 at L = 4096 and D = 64
    assert "attn_mv_c512_h16_f4_l4096.npz" in names and "attn_mv_c1024_h16_f4_l256.npz" in names
    # BASELINE config 4's three MVAttention levels exactly (num_frames = 6: L = 9600 at C = 512, 2400 and 600 at 1024)
    assert {"attn_mv_c512_h16_f6_l9600.npz", "attn_mv_c1024_h16_f6_l2400.npz", "attn_mv_c1024_h16_f6_l600.npz"} <= set(names)


@pytest.mark.parametrize("path", GOLDEN, ids=lambda p: os.path.basename(p)[5:-4])
def test_oracle_reproduces_reference(path):
    """The fp32 restatement reproduces the reference modules' outputs and gradients."""
    meta, z, params, grads = _load(path)
    p = {k: v.clone().requires_grad_(True) for k, v in params.items()}
    x = torch.from_numpy(z["x"]).requires_grad_(True)
    y = _oracle_fn(meta, params)(x, p)
    y.backward(torch.from_numpy(z["gy"]))
    assert _err(y.detach().numpy(), z["y"]) < 1e-6
    assert _err(x.grad.numpy(), z["dx"]) < 1e-5
    for k, g in grads.items():
        assert _err(p[k].grad.numpy(), g) < 1e-5, k


@pytest.mark.parametrize("path", GOLDEN, ids=lambda p: os.path.basename(p)[5:-4])
def test_state_dict_compatible(path):
    """Same submodule / parameter names and shapes as the reference module: its state_dict loads strictly."""
    meta, z, params, _ = _load(path)
    m = _module(meta)
    m.load_state_dict(params, strict=True)


def test_cpu_tensors_take_the_torch_path():
    """CPU tensors (BASELINE config 1) run lgm_amd/cpu.py's torch attention, not the HIP library."""
    from lgm_amd.attention import MemEffAttention
    m = MemEffAttention(64, 2)
    x = torch.randn(1, 8, 64)
    qkv = m.qkv(x).reshape(1, 8, 3, 2, 32)
    ref = ref_attention_core(qkv)
    assert rel_l2(m(x).detach().numpy(), m.proj(ref).detach().numpy()) < 1e-5


def ref_attention_core(qkv):
    q, k, v = (qkv[:, :, i].transpose(1, 2) for i in range(3))
    return ref.attention_core(q, k, v, qkv.shape[-1] ** -0.5).transpose(1, 2).reshape(qkv.shape[0], qkv.shape[1], -1)


# ------------------------------------------------------------------------------------------------------------ GPU
def _packed_truth(qkv, scale, d_o):
    """fp64 softmax attention and its gradient wrt packed qkv [B, L, 3, H, D]."""
    x = qkv.detach().double().requires_grad_(True)
    q, k, v = (x[:, :, i].transpose(1, 2) for i in range(3))
    o = ref.attention_core(q, k, v, scale).transpose(1, 2)
    o.backward(d_o.double())
    return o.detach(), x.grad


@pytest.mark.gpu
@pytest.mark.parametrize("path", GOLDEN, ids=lambda p: os.path.basename(p)[5:-4])
def test_module_matches_reference_fp32(cuda, path):
    meta, z, params, grads = _load(path)
    m = _module(meta).to(cuda)
    m.load_state_dict(params, strict=True)
    x = torch.from_numpy(z["x"]).to(cuda).requires_grad_(True)
    y = m(x)
    y.backward(torch.from_numpy(z["gy"]).to(cuda))
    torch.cuda.synchronize()
    assert _err(y.detach().cpu().numpy(), z["y"]) < 1e-4
    assert _err(x.grad.cpu().numpy(), z["dx"]) < 1e-4
    named = dict(m.named_parameters())
    for k, g in grads.items():
        assert _err(named[k].grad.cpu().numpy(), g) < 1e-4, k


@pytest.mark.gpu
@pytest.mark.parametrize("path", [p for p in GOLDEN if "_mv_" in p], ids=lambda p: os.path.basename(p)[5:-4])
def test_module_bf16_autocast(cuda, path):
    """LGM trains under bf16 mixed precision: the qkv Linear emits bf16 and the kernel runs in bf16."""
    meta, z, params, grads = _load(path)
    m = _module(meta).to(cuda)
    m.load_state_dict(params, strict=True)
    x = torch.from_numpy(z["x"]).to(cuda).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    y.float().backward(torch.from_numpy(z["gy"]).to(cuda))
    assert _err(y.detach().float().cpu().numpy(), z["y"]) < 3e-2
    assert _err(x.grad.float().cpu().numpy(), z["dx"]) < 5e-2


MVA_CASES = [  # C, heads, frames, H, W, batch -- LGM levels (D = 32 / 64) and ragged ones (Cg = 3: scalar stores)
    # the LGM-shaped cases run the register-slab GroupNorm (k_mva_gn_reg) and the vector-access layout kernels;
    # (96, ..., 7, 5) their scalar forms (HW % 4 != 0, Cg % 8 != 0) and the LDS-slab GroupNorm's scalar branches;
    # 46 x 46 at Cg = 16 the LDS-slab GroupNorm's vector path (1,058 items > 1,024; slab 135,552 B <= 144 KB);
    # 48 x 48 at Cg = 16 the chunked fallback (slab 147,584 B > 144 KB: k_mva_stats + k_mva_norm); C = 512 in one
    # group (Cg = 512: no register slab) the LDS slab and k_mva_gn_coef's channel loop (more channels than threads)
    (512, 16, 6, 16, 16, 1), (1024, 16, 6, 10, 10, 1), (256, 8, 4, 8, 8, 2), (96, 3, 2, 7, 5, 1),
    (512, 16, 1, 46, 46, 1), (512, 16, 1, 48, 48, 1), (512, 16, 2, 4, 4, 1, 1)]
# the GroupNorm -> tokens kernel each case must launch (KernelProfiler names, mvattn.hip launch_norm)
MVA_GN_KERNEL = {(512, 16, 6, 16, 16, 1): "k_mva_gn_reg", (1024, 16, 6, 10, 10, 1): "k_mva_gn_reg",
                 (256, 8, 4, 8, 8, 2): "k_mva_gn_reg", (96, 3, 2, 7, 5, 1): "k_mva_gn_tok",
                 (512, 16, 1, 46, 46, 1): "k_mva_gn_tok", (512, 16, 1, 48, 48, 1): "k_mva_stats",
                 (512, 16, 2, 4, 4, 1, 1): "k_mva_gn_tok"}


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["f32", "bf16_autocast"])
@pytest.mark.parametrize("case", MVA_CASES, ids=lambda c: "x".join(map(str, c)))
def test_mvattention_fused_layout_matches_torch_ops(cuda, case, mode):
    """MVAttention's fused GroupNorm->tokens and tokens->residual kernels (lgm_mva_*) and their fused backward
    (lgm_mva_tokens_out_backward, lgm_mva_norm_tokens_backward) against the same module on upstream's torch ops
    (fused=False): forward, dL/dx and the GroupNorm / Linear parameter gradients. fp32: the only difference is the
    order of the GroupNorm sums (1e-5, forward and gradients); bf16: tokens may round to neighbouring bf16 values
    (1e-2; gradients 1e-1). The fused backward's sums run in a fixed order: two runs are bitwise equal."""
    from lgm_amd import _native
    from lgm_amd.attention import MVAttention
    C, heads, frames, H, W, B = case[:6]
    groups = case[6] if len(case) > 6 else 32
    torch.manual_seed(11)
    m = MVAttention(C, heads, num_frames=frames, skip_scale=0.5 ** 0.5, groups=groups).to(cuda)
    with torch.no_grad():
        m.norm.weight.uniform_(0.5, 1.5)
        m.norm.bias.uniform_(-0.2, 0.2)
    x0 = torch.randn(B * frames, C, H, W, device=cuda) * 2 + 0.3
    gy = torch.randn(B * frames, C, H, W, device=cuda)
    outs = []
    prof = _native.KernelProfiler()
    for fused in (True, True, False):
        m.fused = fused
        m.zero_grad()
        x = x0.clone().requires_grad_(True)
        with prof:
            if mode == "f32":
                y = m(x)
            else:
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    y = m(x)
            y.float().backward(gy)
        if fused:
            ran = prof.summary()
            prof.reset()
            gn = {k for k in ran if k in ("k_mva_gn_reg", "k_mva_gn_tok", "k_mva_stats")}
            assert gn == {MVA_GN_KERNEL[case]}, (case, sorted(ran))
            assert "k_mva_gn_coef" in ran and "k_mva_out" in ran, sorted(ran)
        outs.append((y.dtype, y.detach().float(), x.grad.float(), {k: p.grad.float() for k, p in m.named_parameters()}))
    prof.close()
    tol, gtol = (1e-5, 1e-5) if mode == "f32" else (1e-2, 1e-1)
    (tf, yf, dxf, gf), (_, yf2, dxf2, gf2), (tt, yt, dxt, gt) = outs
    assert tf == tt
    assert torch.equal(yf, yf2) and torch.equal(dxf, dxf2) and all(torch.equal(gf[k], gf2[k]) for k in gf)
    errs = {"y": rel_l2(yf.cpu().numpy(), yt.cpu().numpy()), "dx": rel_l2(dxf.cpu().numpy(), dxt.cpu().numpy())}
    errs.update({k: rel_l2(gf[k].cpu().numpy(), gt[k].cpu().numpy()) for k in gt})
    print(f"mva fused vs torch ops {case} {mode}: " + ", ".join(f"{k} {v:.2e}" for k, v in errs.items()))
    assert errs["y"] < tol
    for k, e in errs.items():
        assert e < gtol, (k, e)


SHAPES = [  # B, L, H, D -- LGM levels (4 views x 8^2 / 16^2 / 32^2 tokens, D = 64 / 64 / 32) and ragged edges
    (1, 256, 16, 64), (2, 1024, 16, 64), (1, 4096, 16, 32), (1, 1, 2, 32), (3, 65, 2, 64), (2, 100, 3, 128),
    (1, 17, 1, 32), (2, 600, 4, 32), (2, 4100, 16, 32),  # the last one: two query sub-tiles per wave + a tail
    # LGM 'big' (BASELINE config 4: 6 input views at 320, core/unet.py:35-49): L = 6 x 40^2 at C = 512 (D = 32),
    # 6 x 20^2 and 6 x 10^2 at C = 1024 (D = 64)
    (1, 9600, 16, 32), (1, 2400, 16, 64), (1, 600, 16, 64),
    # D = 64 with two query sub-tiles per wave (ceil(L/128) * B * H >= 512): LGM's default training level
    # (B = 8 is sharded; 4 x 1024 crosses the threshold) and the 'big' 2400-token level at B = 2
    (4, 1024, 16, 64), (2, 2400, 16, 64),
    # D = 32 with FOUR query sub-tiles per forward wave (ceil(L/256) * B * H >= 1,536 workgroups: LGM training's
    # B = 8 x L 4096 level) and a partial last tile: 17 x 96 = 1,632 workgroups
    (6, 4100, 16, 32),
]


def _sdpa_errors(qkv, scale, d_o, o_t, dqkv_t, floor):
    """The same 16-bit inputs through torch's own attention (F.scaled_dot_product_attention, whichever ROCm backend
    torch picks) against the same fp64 truth: an independent measure of what the format allows on these inputs, so
    the 16-bit bars are pinned to a baseline rather than to this kernel."""
    import torch.nn.functional as F
    x = qkv.clone().requires_grad_(True)
    q, k, v = (x[:, :, i].transpose(1, 2) for i in range(3))
    o = F.scaled_dot_product_attention(q, k, v, scale=scale).transpose(1, 2)
    o.backward(d_o)
    torch.cuda.synchronize()
    out = {"o": rel_l2(o.detach().double().cpu().numpy(), o_t.cpu().numpy())}
    for i, name in enumerate("qkv"):
        a, b = x.grad[:, :, i].double(), dqkv_t[:, :, i]
        out["d" + name] = float((a - b).norm()) / max(float(b.norm()), floor)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 2e-2), (torch.float16, 3e-3)],
                         ids=["f32", "bf16", "f16"])
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_packed_attention_vs_fp64(cuda, shape, dtype, tol):
    from lgm_amd.attention import packed_attention
    B, L, H, D = shape
    g = torch.Generator(device="cpu").manual_seed(B * 7919 + L * 31 + H * 7 + D)
    qkv = (torch.randn((B, L, 3, H, D), generator=g) * 1.5).to(cuda, dtype)
    d_o = torch.randn((B, L, H, D), generator=g).to(cuda, dtype)
    scale = D ** -0.5
    x = qkv.clone().requires_grad_(True)
    o = packed_attention(x, scale)
    o.backward(d_o)
    o = o.detach()
    torch.cuda.synchronize()
    o_t, dqkv_t = _packed_truth(qkv, scale, d_o)
    assert o.dtype == dtype and x.grad.dtype == dtype
    assert torch.isfinite(o).all() and torch.isfinite(x.grad).all()
    # per-slice relative L2, normalised by at least 1% of the whole dqkv norm: with L = 1 the softmax is constant
    # and the true dq is exactly 0 (only rounding noise of dP - delta remains)
    floor = 1e-2 * float(dqkv_t.norm())
    errs = {"o": rel_l2(o.double().cpu().numpy(), o_t.cpu().numpy())}
    for i, name in enumerate("qkv"):
        a, b = x.grad[:, :, i].double(), dqkv_t[:, :, i]
        errs["d" + name] = float((a - b).norm()) / max(float(b.norm()), floor)
    sd = _sdpa_errors(qkv, scale, d_o, o_t, dqkv_t, floor) if dtype != torch.float32 else None
    print(f"attention vs fp64 {shape} {dtype}: " + ", ".join(
        f"{k} {v:.2e}" + (f" (sdpa {sd[k]:.2e})" if sd else "") for k, v in errs.items()))
    for k, e in errs.items():
        assert e < tol, (k, e)
        if sd is not None:
            # 16-bit: against torch's own attention on the same inputs (an independent baseline). Measured
            # (profiles/r06/attn_vs_sdpa): o 2.0-2.25x, dq / dk / dv 1.3-1.85x SDPA's error. The excess is ONE
            # deliberate rounding: the kernels pre-multiply Q by scale * log2(e) in 16 bits (the softmax scale then
            # rides on the MFMA instead of one VALU op per score, -15 % attention time), which
            # perturbs every score by ~2^-9 relative (sqrt(1 + 2^2) ~ 2.2x SDPA's output-rounding-dominated error).
            # Held at 2.5x SDPA so any other precision loss shows.
            assert e <= max(2.5 * sd[k], tol / 8), (k, e, sd[k])


@pytest.mark.gpu
@pytest.mark.parametrize("jump", [6.0, 30.0, 100.0, -100.0])
@pytest.mark.parametrize("dtype,tol", [(torch.bfloat16, 2e-2), (torch.float16, 3e-3)], ids=["bf16", "f16"])
@pytest.mark.parametrize("D", [32, 64])
def test_forward_score_jump(cuda, D, dtype, tol, jump):
    """The forward's online softmax where one key of a LATER key tile scores `jump` (log2 units) above every key of
    the first tile, for every query (or, negative, far below): the paths that raise the row reference m mid-row
    (rare on bounded random data, so pinned here) must give the fp64 result. With a near-one-hot softmax
    dS = P (dP - delta) is a cancellation that amplifies the 16-bit rounding of the inputs and of the stored output,
    so the gradients are held to the fixed bar OR to 1.25x the error of torch's own attention
    (F.scaled_dot_product_attention) on the same 16-bit inputs against the same fp64 truth -- a bar set by an
    independent implementation, not by this kernel."""
    from lgm_amd.attention import packed_attention
    B, L, H = 1, 320, 2
    scale = D ** -0.5
    g = torch.Generator(device="cpu").manual_seed(int(abs(jump)) * 13 + D + (1 if jump < 0 else 0))
    c = torch.full((D,), 0.5)
    qkv = torch.randn((B, L, 3, H, D), generator=g) * 0.3
    qkv[:, :, 0] += c  # every query ~ c
    # key 200 (the fourth 64-key tile) scores ~ jump (log2 units) above the others for every query
    beta = jump / (1.4426950408889634 * scale * float(c @ c))
    qkv[:, 200, 1] = beta * c
    qkv = qkv.to(cuda, dtype)
    d_o = torch.randn((B, L, H, D), generator=g).to(cuda, dtype)
    x = qkv.clone().requires_grad_(True)
    o = packed_attention(x, scale)
    o.backward(d_o)
    o = o.detach()
    torch.cuda.synchronize()
    o_t, dqkv_t = _packed_truth(qkv, scale, d_o)
    assert torch.isfinite(o).all() and torch.isfinite(x.grad).all()
    assert rel_l2(o.double().cpu().numpy(), o_t.cpu().numpy()) < tol
    floor = 1e-2 * float(dqkv_t.norm())
    sd = _sdpa_errors(qkv, scale, d_o, o_t, dqkv_t, floor)
    for i, name in enumerate("qkv"):
        a, b = x.grad[:, :, i].double(), dqkv_t[:, :, i]
        err = float((a - b).norm()) / max(float(b.norm()), floor)
        print(f"score jump {jump} D {D} {dtype} d{name}: {err:.2e} (sdpa {sd['d' + name]:.2e})")
        assert err <= max(tol, 1.25 * sd["d" + name]), (name, err, sd["d" + name])


@pytest.mark.gpu
def test_memory_efficient_attention_views_and_copies(cuda):
    """xformers-style entry: unbind views of the packed tensor run in place; unrelated q/k/v are stacked."""
    from lgm_amd.attention import memory_efficient_attention
    B, L, H, D = 2, 130, 4, 32
    qkv = torch.randn(B, L, 3, H, D, device=cuda)
    q, k, v = torch.unbind(qkv, 2)
    o1 = memory_efficient_attention(q, k, v)
    o2 = memory_efficient_attention(q.contiguous(), k.contiguous(), v.contiguous())
    assert torch.equal(o1, o2)
    o_t, _ = _packed_truth(qkv, D ** -0.5, torch.zeros(B, L, H, D, device=cuda))
    assert rel_l2(o1.double().cpu().numpy(), o_t.cpu().numpy()) < 1e-4


@pytest.mark.gpu
def test_attention_deterministic(cuda):
    from lgm_amd.attention import packed_attention
    qkv = torch.randn(1, 1024, 3, 16, 64, device=cuda, dtype=torch.bfloat16)
    d_o = torch.randn(1, 1024, 16, 64, device=cuda, dtype=torch.bfloat16)
    outs = []
    for _ in range(2):
        x = qkv.clone().requires_grad_(True)
        o = packed_attention(x)
        o.backward(d_o)
        outs.append((o, x.grad))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("where", ["q", "k", "v"])
def test_nan_propagates_like_sdpa(cuda, dtype, where):
    """A NaN anywhere in q/k/v reaches the output and the gradients exactly where torch's attention puts it (the
    divergence detection of a bf16 training run relies on NaN propagation; attention.hip is built without IEEE NaN
    semantics for its max / exp chains, so this pins that no NaN is dropped): NaN masks of o and of dqkv equal
    those of the fp32 torch math on the same inputs."""
    from lgm_amd.attention import packed_attention
    B, L, H, D = 2, 200, 2, 32
    gen = torch.Generator().manual_seed(9)
    qkv = torch.randn(B, L, 3, H, D, generator=gen)
    qkv[1, 37, "qkv".index(where), 1, 5] = float("nan")
    d_o = torch.randn(B, L, H, D, generator=gen)
    x = qkv.to(cuda, dtype).requires_grad_(True)
    o = packed_attention(x)
    o.backward(d_o.to(cuda, dtype))
    torch.cuda.synchronize()
    xr = qkv.clone().requires_grad_(True)
    q, k, v = (xr[:, :, i].transpose(1, 2) for i in range(3))
    p = torch.softmax((q * D ** -0.5) @ k.transpose(-1, -2), dim=-1)
    orf = (p @ v).transpose(1, 2)
    orf.backward(d_o)
    assert torch.isnan(orf).any()
    assert torch.equal(torch.isnan(o.float().cpu()), torch.isnan(orf)), "output NaN pattern differs"
    assert torch.equal(torch.isnan(x.grad.float().cpu()), torch.isnan(xr.grad)), "gradient NaN pattern differs"


# measured (profiles/r05/attn_prescale, seeded inputs of test_packed_attention_vs_fp64, rel L2 vs fp64) x 1.25: with
# every kernel recomputing P from the same rounded Q * scale * log2(e), dK / dV sit beside o / dQ (the K * c form of
# round 4 left them at 7.2e-3 in bf16, 9.2e-4 in fp16)
ERROR_RECORD = {torch.bfloat16: {"o": 3.96e-3, "dq": 4.30e-3, "dk": 4.47e-3, "dv": 4.08e-3},
                torch.float16: {"o": 5.00e-4, "dq": 5.46e-4, "dk": 5.65e-4, "dv": 5.19e-4}}


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
def test_attention_error_record_d32(cuda, dtype):
    """Kernel-level parity of the 16-bit path at LGM's D = 32 bench level (L 4096, 16 heads): o, dq, dk, dv each
    within 1.25x of its recorded error against fp64 -- a regression of any one kernel's rounding shows up here, far
    below the 2e-2 / 3e-3 bars of test_packed_attention_vs_fp64."""
    from tests.attn_precision import errors
    e = errors(cuda, (1, 4096, 16, 32), dtype)
    print(f"attention error record {dtype}: " + ", ".join(f"{k} {v:.3e}" for k, v in e.items()))
    for k, v in e.items():
        assert v <= 1.25 * ERROR_RECORD[dtype][k], (k, v)
