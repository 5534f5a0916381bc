"""The weight-gradient GEMM of MVAttention's Linears (include/lgm_linear.h, lgm_amd/csrc/wgrad.hip) against fp64, and
the module path that uses it (lgm_amd/linear.py) against torch's own autograd through nn.Linear under bf16 autocast
(core/attention.py:46,48: the qkv and proj projections of MemEffAttention)."""
import numpy as np
import pytest
import torch

from lgm_amd import _native

# K, M, N, ld_dy (0: M), bias -- the bench's MVAttention level (8 objects x 4 views x 32^2 tokens, C = 512: qkv and
# proj), LGM 'big' cfg4 levels (K = 9,600 / 2,400 / 600 tokens, C = 512 / 1024), and ragged edges: K not a multiple
# of the 64-row stage, M / N not multiples of the 128 tile, K = 0, a strided dy (a column slice of a wider tensor)
WG_CASES = [(32768, 1536, 512, 0, False), (32768, 512, 512, 0, True), (9600, 1536, 512, 0, False),
            (2400, 3072, 1024, 0, False), (600, 1024, 1024, 0, True), (1234, 200, 136, 0, True), (33, 8, 8, 0, True),
            (0, 64, 64, 0, True), (777, 96, 40, 160, True), (5, 24, 16, 0, False)]


def _ref(dy, x):
    d, xx = dy.double(), x.double()
    return d.t() @ xx, d.sum(0)


def _wgrad(dy, x, want_db, ld_dy=None):
    L = _native.lib()
    K, N = x.shape
    M = dy.shape[1]
    ld = ld_dy or dy.stride(0)
    code = {torch.bfloat16: 1, torch.float16: 2}[dy.dtype]
    dw = torch.full((M, N), float("nan"), device=dy.device)
    db = torch.full((M,), float("nan"), device=dy.device) if want_db else None
    ws_bytes = L.lgm_linear_wgrad_workspace_size(K, M, N, int(want_db))
    ws = torch.empty(max(ws_bytes, 1), device=dy.device, dtype=torch.uint8)
    _native.check(L.lgm_linear_wgrad(code, K, M, N, _native.ptr(dy), ld, _native.ptr(x), x.stride(0), _native.ptr(dw),
                                     _native.ptr(db), _native.ptr(ws), ws_bytes, _native.stream_of(dy.device), None),
                  "lgm_linear_wgrad")
    torch.cuda.synchronize()
    return dw, db


def test_workspace_size_and_errors():
    L = _native.lib()
    assert L.lgm_linear_wgrad_workspace_size(32768, 1536, 512, 0) > 0
    assert L.lgm_linear_wgrad_workspace_size(32768, 512, 512, 1) > L.lgm_linear_wgrad_workspace_size(32768, 512, 512, 0)
    assert L.lgm_linear_wgrad_workspace_size(10, 0, 8, 0) == 0
    rc = L.lgm_linear_wgrad(0, 16, 8, 8, None, 8, None, 8, None, None, None, 0, None, None)  # fp32: not this kernel
    assert rc < 0 and b"dtype" in L.lgm_last_error()
    rc = L.lgm_linear_wgrad(1, 16, 12, 8, None, 12, None, 8, None, None, None, 0, None, None)
    assert rc < 0 and b"multiples of 8" in L.lgm_last_error()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("case", WG_CASES, ids=lambda c: "x".join(map(str, c[:4])) + ("b" if c[4] else ""))
def test_wgrad_vs_fp64(cuda, case, dtype):
    """dw = dy^T x and db = colsum(dy) vs fp64 on the same 16-bit operands: the products are exact and the sums fp32,
    so the error is fp32 summation noise (rel L2 < 1e-5); two runs are bitwise equal (fixed split order)."""
    K, M, N, ld, want_db = case
    g = torch.Generator().manual_seed(K * 7 + M * 3 + N)
    wide = torch.randn((K, ld or M), generator=g).to(cuda, dtype)
    dy = wide[:, :M]
    x = torch.randn((K, N), generator=g).to(cuda, dtype)
    dw, db = _wgrad(dy, x, want_db, ld_dy=ld or M)
    dw2, db2 = _wgrad(dy, x, want_db, ld_dy=ld or M)
    rw, rb = _ref(dy, x)
    assert torch.isfinite(dw).all()
    assert torch.equal(dw, dw2) and (db is None or torch.equal(db, db2))
    if K == 0:
        assert torch.all(dw == 0) and (db is None or torch.all(db == 0))
        return
    e = float((dw.double() - rw).norm() / rw.norm())
    print(f"wgrad {case} {dtype}: dw rel L2 {e:.2e}" + (f", db {float((db.double() - rb).norm() / rb.norm()):.2e}"
                                                        if want_db else ""))
    assert e < 1e-5
    if want_db:
        assert float((db.double() - rb).norm() / rb.norm()) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("bias", [False, True])
def test_linear16_matches_torch_autocast(cuda, bias):
    """lgm_amd.linear.linear under bf16 autocast: forward and input gradient bitwise torch's (the same library GEMMs);
    weight / bias gradients = torch's to its bf16 rounding (torch rounds its bf16 dW before the fp32 cast: 2^-9
    relative per element, ~2e-3 rel L2), and closer to the fp64 truth than torch's."""
    from lgm_amd.linear import linear
    torch.manual_seed(1)
    lin = torch.nn.Linear(512, 1536, bias=bias).to(cuda)
    x0 = torch.randn(4, 1024, 512, device=cuda)
    gy = torch.randn(4, 1024, 1536, device=cuda)
    outs = []
    for native in (True, False):
        lin.zero_grad()
        x = x0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = linear(x, lin) if native else lin(x)
        y.float().backward(gy)
        outs.append((y.detach(), x.grad.clone(), lin.weight.grad.clone(), None if not bias else lin.bias.grad.clone()))
    (yn, dxn, dwn, dbn), (yt, dxt, dwt, dbt) = outs
    assert yn.dtype == yt.dtype == torch.bfloat16
    assert torch.equal(yn, yt) and torch.equal(dxn, dxt)
    x16 = x0.to(torch.bfloat16).reshape(-1, 512)
    g16 = gy.to(torch.bfloat16).reshape(-1, 1536)
    rw, rb = _ref(g16, x16)
    e_n = float((dwn.double() - rw).norm() / rw.norm())
    e_t = float((dwt.double() - rw).norm() / rw.norm())
    print(f"linear16 dW vs fp64: native {e_n:.2e}, torch {e_t:.2e}")
    assert e_n < 1e-5 and e_n <= e_t
    assert float((dwn - dwt).norm() / dwt.norm()) < 5e-3
    if bias:
        assert float((dbn.double() - rb).norm() / rb.norm()) < 1e-5
        assert float((dbn - dbt).norm() / dbt.norm()) < 5e-3


@pytest.mark.gpu
def test_linear16_inference_is_plain_linear(cuda, monkeypatch):
    """Without a graph to record (no_grad, or nothing requiring grad) linear() is lin(x) itself: bitwise torch's
    autocast output, and the autograd Function (its host cost and weight cast per call) is never entered."""
    from lgm_amd import linear as LN

    def boom(*a, **k):
        raise AssertionError("_Linear16 used without a graph")

    lin = torch.nn.Linear(512, 1536).to(cuda)
    x = torch.randn(2, 256, 512, device=cuda)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ref = lin(x)
        monkeypatch.setattr(LN._Linear16, "apply", boom)
        with torch.no_grad():
            assert torch.equal(LN.linear(x, lin), ref)
        lin.requires_grad_(False)
        assert torch.equal(LN.linear(x, lin), ref)


@pytest.mark.gpu
def test_mvattention_uses_native_wgrad(cuda):
    """MVAttention under bf16 autocast (the bench's level shape, 1 object): k_wgrad runs for both Linears, and the
    parameter gradients match the upstream autograd path (native_wgrad = False) to torch's bf16 rounding."""
    from lgm_amd.attention import MVAttention
    torch.manual_seed(4)
    m = MVAttention(512, 16, num_frames=4, skip_scale=0.5 ** 0.5).to(cuda)
    x0 = torch.randn(4, 512, 32, 32, device=cuda)
    gy = torch.randn(4, 512, 32, 32, device=cuda)
    grads = []
    for native in (True, False):
        m.attn.native_wgrad = native
        m.zero_grad()
        prof = _native.KernelProfiler()
        with prof:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = m(x0)
            y.float().backward(gy)
        ran = prof.summary()
        prof.close()
        assert ("k_wgrad" in ran) == native and (not native or ran["k_wgrad"][0] == 2), ran
        grads.append({k: p.grad.clone() for k, p in m.named_parameters()})
    for k in ("attn.qkv.weight", "attn.proj.weight", "attn.proj.bias"):
        e = float((grads[0][k] - grads[1][k]).norm() / grads[1][k].norm())
        assert e < 1e-2, (k, e)
