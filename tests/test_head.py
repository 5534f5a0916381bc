"""Fused Gaussian head (lgm_amd/head.py, include/lgm_head.h): LGM.forward_gaussians' epilogue
(core/models.py:95-117) against its fp32 torch restatement (oracle/head_ref.py), forward and backward.

Tolerances (floating point): Gaussians and all gradients (dx, d_weight, d_bias) within max(1e-5, 1.25 x the fp32
restatement's own error) relative L2 of the restatement evaluated in fp64, for fp32 input; bf16 input: the same bf16 values fed to the restatement in fp32, dx compared
after bf16 rounding (2e-3). The kernels accumulate in a fixed order: two backward runs are bitwise identical."""
import numpy as np
import pytest
import torch

from lgm_amd import _native
from lgm_amd.head import GaussianHead, gaussian_head
from oracle.head_ref import forward_gaussians_epilogue
from tests.render_cases import GRAD_FACTOR, rel_l2


def _inputs(B, V, h, w, seed, dtype=torch.float32):
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(B * V, 14, h, w, generator=g) * 1.5).to(dtype)
    conv = torch.nn.Conv2d(14, 14, 1)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(14, 14, 1, 1, generator=g) * 0.6)
        conv.bias.copy_(torch.randn(14, generator=g))
        conv.bias[5] = 21.0  # softplus above its threshold (20) on most points
        conv.bias[0] = 0.8   # pos partly beyond the clamp
    d = torch.randn(B, V * h * w, 14, generator=g)
    return x, conv, d


def test_module_api_cpu():
    m = GaussianHead()
    assert set(m.state_dict()) == {"conv.weight", "conv.bias"}  # LGM's self.conv (core/models.py:34)
    x = torch.randn(4, 14, 2, 3)
    # CPU tensors (BASELINE config 1): the torch path of lgm_amd/cpu.py
    ref = forward_gaussians_epilogue(x, m.conv.weight, m.conv.bias, 1, 4)
    assert rel_l2(m(x, 1, 4).detach().numpy(), ref.detach().numpy()) < 1e-6


def test_restatement_matches_reference_semantics():
    """The oracle's rotation is F.normalize's default dim=1 on the [B, N, 4] slice (core/models.py:43,112)."""
    x, conv, _ = _inputs(2, 3, 4, 5, seed=1)
    out = forward_gaussians_epilogue(x, conv.weight, conv.bias, 2, 3)
    assert out.shape == (2, 60, 14)
    np.testing.assert_allclose(out[..., 7:11].norm(dim=1).detach().numpy(), 1.0, rtol=1e-5)


def _torch_ref(x, conv, d, B, V, dtype):
    xr = x.to(dtype).clone().requires_grad_(True)
    cr = torch.nn.Conv2d(14, 14, 1).to(dtype)
    cr.load_state_dict({k: v.to(dtype) for k, v in conv.state_dict().items()})
    out = forward_gaussians_epilogue(xr, cr.weight, cr.bias, B, V)
    out.backward(d.to(dtype))
    return {"out": out.detach().numpy(), "dx": xr.grad.numpy(), "dW": cr.weight.grad.numpy(),
            "db": cr.bias.grad.numpy()}


@pytest.mark.gpu
@pytest.mark.parametrize("B,V,h,w", [(1, 4, 64, 64), (2, 3, 17, 23), (1, 6, 160, 160), (3, 1, 1, 1)])
def test_head_fp32_vs_torch(cuda, B, V, h, w):
    """GPU vs the restatement evaluated in fp64, bar max(1e-5, 1.25 x the fp32 restatement's own error, the render
    tests' GRAD_FACTOR): the
    rotation's normalisation over N Gaussians (a 153,600-term sum at cfg4) leaves torch's fp32 CPU reduction
    ~1.4e-5 off, so the fp32 restatement cannot be the bar there."""
    x, conv, d = _inputs(B, V, h, w, seed=B * 100 + V * 10 + h)
    r32 = _torch_ref(x, conv, d, B, V, torch.float32)
    r64 = _torch_ref(x, conv, d, B, V, torch.float64)
    xg = x.to(cuda).requires_grad_(True)
    cg = torch.nn.Conv2d(14, 14, 1).to(cuda)
    cg.load_state_dict(conv.state_dict())
    out = gaussian_head(xg, cg, B, V)
    out.backward(d.to(cuda))
    torch.cuda.synchronize()
    assert tuple(out.shape) == r64["out"].shape and out.dtype == torch.float32
    gpu = {"out": out.detach().cpu().numpy(), "dx": xg.grad.cpu().numpy(), "dW": cg.weight.grad.cpu().numpy(),
           "db": cg.bias.grad.cpu().numpy()}

    def check(name, a, b32, b64):
        e32 = rel_l2(b32, b64)
        bar = max(1e-5, GRAD_FACTOR * e32)
        e = rel_l2(a, b64)
        print(f"head {B}x{V}x{h}x{w} {name}: GPU {e:.3e}, fp32 restatement {e32:.3e}, bar {bar:.3e}")
        assert e < bar, f"{name}: GPU vs fp64 {e:.3e}, bar {bar:.3e}"

    for k in gpu:
        check(k, gpu[k], r32[k], r64[k])
    for sl in (slice(0, 3), slice(3, 4), slice(4, 7), slice(7, 11), slice(11, 14)):  # each activation on its own
        check(f"out[{sl}]", gpu["out"][..., sl], r32["out"][..., sl], r64["out"][..., sl])


@pytest.mark.gpu
def test_head_bf16_input(cuda):
    B, V, h, w = 2, 6, 40, 40
    x, conv, d = _inputs(B, V, h, w, seed=7, dtype=torch.bfloat16)
    xr = x.float().clone().requires_grad_(True)  # the same bf16 values, fp32 arithmetic
    ref = forward_gaussians_epilogue(xr, conv.weight, conv.bias, B, V)
    ref.backward(d)
    cg = torch.nn.Conv2d(14, 14, 1).to(cuda)
    cg.load_state_dict(conv.state_dict())
    xg = x.to(cuda).requires_grad_(True)
    out = gaussian_head(xg, cg, B, V)
    out.backward(d.to(cuda))
    assert xg.grad.dtype == torch.bfloat16
    assert rel_l2(out.detach().cpu().numpy(), ref.detach().numpy()) < 1e-5
    assert rel_l2(xg.grad.float().cpu().numpy(), xr.grad.bfloat16().float().numpy()) < 2e-3
    assert rel_l2(cg.weight.grad.cpu().numpy(), conv.weight.grad.numpy()) < 1e-5
    assert rel_l2(cg.bias.grad.cpu().numpy(), conv.bias.grad.numpy()) < 1e-5


@pytest.mark.gpu
def test_head_backward_deterministic(cuda):
    x, conv, d = _inputs(1, 6, 160, 160, seed=3)
    cg = conv.to(cuda)
    grads = []
    for _ in range(2):
        xg = x.to(cuda).requires_grad_(True)
        cg.zero_grad()
        gaussian_head(xg, cg, 1, 6).backward(d.to(cuda))
        grads.append((xg.grad.clone(), cg.weight.grad.clone(), cg.bias.grad.clone()))
    for a, b in zip(*grads):
        assert torch.equal(a, b)
