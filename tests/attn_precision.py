"""Per-output error of the packed attention kernels against fp64 (shared by tests/test_attention.py and
scripts/diag_attn_precision.py)."""
import torch

from oracle import attention_ref as ref


def seeded_qkv(shape, dtype, device):
    """test_packed_attention_vs_fp64's inputs: qkv ~ 1.5 N(0, 1) [B, L, 3, H, D] and d_o ~ N(0, 1), seeded by shape."""
    B, L, H, D = shape
    g = torch.Generator(device="cpu").manual_seed(B * 7919 + L * 31 + H * 7 + D)
    qkv = (torch.randn((B, L, 3, H, D), generator=g) * 1.5).to(device, dtype)
    d_o = torch.randn((B, L, H, D), generator=g).to(device, dtype)
    return qkv, d_o


def packed_truth(qkv, scale, d_o):
    """fp64 softmax attention and its gradient wrt packed qkv [B, L, 3, H, D]."""
    x = qkv.detach().double().requires_grad_(True)
    q, k, v = (x[:, :, i].transpose(1, 2) for i in range(3))
    o = ref.attention_core(q, k, v, scale).transpose(1, 2)
    o.backward(d_o.double())
    return o.detach(), x.grad


def errors(device, shape, dtype):
    """{'o', 'dq', 'dk', 'dv'}: relative L2 of the HIP kernels' outputs vs fp64 on the same rounded inputs."""
    from lgm_amd.attention import packed_attention
    qkv, d_o = seeded_qkv(shape, dtype, device)
    scale = shape[3] ** -0.5
    x = qkv.clone().requires_grad_(True)
    o = packed_attention(x, scale)
    o.backward(d_o)
    torch.cuda.synchronize()
    o_t, g_t = packed_truth(qkv, scale, d_o)  # (fp64 on the GPU: the L 9600 score matrix is 12 GB)

    def rl(a, b):
        return float((a.double() - b).norm() / b.norm())

    out = {"o": rl(o.detach(), o_t)}
    for i, n in enumerate(("dq", "dk", "dv")):
        out[n] = rl(x.grad[:, :, i], g_t[:, :, i])
    return out
