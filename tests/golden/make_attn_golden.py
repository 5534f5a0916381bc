"""Golden vectors for the attention path, produced by the REFERENCE's own modules (run in the survey container
only; /root/reference never travels): core/attention.py MemEffAttention (pure-torch fallback, XFORMERS_DISABLED=1:
core/attention.py:16-28, 51-64) and core/unet.py MVAttention (:11-49). fp32, CPU.

Each case stores: x, upstream grad gy, the module's state_dict (same parameter names as ours), y, dx, and the
parameter gradients. Regenerate with: PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_attn_golden.py

LGM's real widths (core/unet.py:35-49 with 16 heads, core/unet.py:113-206): C = 512 (D = 32) at 4 views x 32^2
(L = 4096, the heaviest 'big' level) and C = 1024 (D = 64) at 4 views x 8^2. Their parameters and inputs would be
tens of MB as arrays, so these "seeded" fixtures store no inputs at all: the parameters, x and gy are drawn from
a CPU torch.Generator (seed = crc32 of the case name) in a fixed order that tests/test_attention.py replays
(seeded_inputs), and of every output (y, dx, each parameter gradient) only a deterministic strided sample of at
most 32,768 elements plus the full array's float64 L2 norm and sum are kept.
"""
import os
import sys
import zlib

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def seeded_inputs(name, param_shapes, x_shape):
    """The seeded fixtures' inputs, drawn in this order from one CPU generator: every parameter (named_parameters()
    order; weights * 0.5 / sqrt(fan_in), vectors * 0.1, the GroupNorm weight + 1), then x, then (returned as a
    function of y's shape) gy. Shared verbatim with tests/test_attention.py, which imports it."""
    g = torch.Generator().manual_seed(zlib.crc32(name.encode()))
    params = {}
    for k, shp in param_shapes:
        t = torch.randn(shp, generator=g) * (0.5 / np.sqrt(shp[-1]) if len(shp) > 1 else 0.1)
        if k == "norm.weight":
            t = t + 1.0
        params[k] = t
    x = torch.randn(x_shape, generator=g)
    return params, x, lambda shape: torch.randn(shape, generator=g)


def sample(a, n=32768):
    """A deterministic strided sample of at most n elements of a flattened array: (indices, values)."""
    flat = a.reshape(-1)
    idx = (np.arange(min(n, flat.size), dtype=np.int64) * 7919 + 13) % flat.size
    return idx.astype(np.int64), flat[idx]


def main():
    os.environ["XFORMERS_DISABLED"] = "1"
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    from core.attention import MemEffAttention  # noqa: E402  (reference code, read-only)
    from core.unet import MVAttention  # noqa: E402

    torch.manual_seed(0)
    # LGM's head dims are 32 (C=512 / 16 heads) and 64 (C=1024 / 16 heads); channel counts are reduced here to
    # keep the fixtures small, token counts L = F*h*w keep LGM's structure (incl. L = 600, not a multiple of 64).
    cases = [
        # name, kind, ctor kwargs, input shape
        ("memeff_d128_h4", "memeff", dict(dim=128, num_heads=4), (2, 200, 128)),
        ("memeff_d128_h2", "memeff", dict(dim=128, num_heads=2), (1, 130, 128)),
        ("mv_c64_h2_f4", "mv", dict(dim=64, num_heads=2, num_frames=4, skip_scale=0.5 ** 0.5), (4, 64, 4, 4)),
        ("mv_c128_h4_f4", "mv", dict(dim=128, num_heads=4, num_frames=4, skip_scale=0.5 ** 0.5), (4, 128, 16, 16)),
        ("mv_c256_h4_f4", "mv", dict(dim=256, num_heads=4, num_frames=4, skip_scale=0.5 ** 0.5), (4, 256, 8, 8)),
        ("mv_c128_h4_f6", "mv", dict(dim=128, num_heads=4, num_frames=6, skip_scale=0.5 ** 0.5), (6, 128, 10, 10)),
        # LGM 'big' (6 input views at 320 -> 20^2 at the D=64 level): L = 6 * 20 * 20 = 2400 tokens at D = 32 and 64
        ("mv_c64_h2_f6_l2400", "mv", dict(dim=64, num_heads=2, num_frames=6, skip_scale=0.5 ** 0.5), (6, 64, 20, 20)),
        ("mv_c128_h2_f6_l2400", "mv", dict(dim=128, num_heads=2, num_frames=6, skip_scale=0.5 ** 0.5),
         (6, 128, 20, 20)),
    ]
    seeded = [  # name, ctor kwargs, input shape: LGM's real channel widths, 16 heads
        ("mv_c512_h16_f4_l4096", dict(dim=512, num_heads=16, num_frames=4, skip_scale=0.5 ** 0.5), (4, 512, 32, 32)),
        ("mv_c1024_h16_f4_l256", dict(dim=1024, num_heads=16, num_frames=4, skip_scale=0.5 ** 0.5), (4, 1024, 8, 8)),
        # BASELINE config 4, LGM 'big' (6 input views at 320, core/unet.py:35-49 with num_frames=6): its three
        # attention levels exactly -- C = 512 at 40^2 (L = 9600, D = 32), C = 1024 at 20^2 (L = 2400) and 10^2 (L = 600)
        ("mv_c512_h16_f6_l9600", dict(dim=512, num_heads=16, num_frames=6, skip_scale=0.5 ** 0.5), (6, 512, 40, 40)),
        ("mv_c1024_h16_f6_l2400", dict(dim=1024, num_heads=16, num_frames=6, skip_scale=0.5 ** 0.5),
         (6, 1024, 20, 20)),
        ("mv_c1024_h16_f6_l600", dict(dim=1024, num_heads=16, num_frames=6, skip_scale=0.5 ** 0.5), (6, 1024, 10, 10)),
    ]
    only = set(sys.argv[1:])  # optional: regenerate only the named cases
    for name, kw, shape in seeded:
        if only and name not in only:
            continue
        m = MVAttention(kw["dim"], kw["num_heads"], num_frames=kw["num_frames"], skip_scale=kw["skip_scale"])
        names = [k for k, _ in m.named_parameters()]
        params, x, draw_gy = seeded_inputs(name, [(k, tuple(p.shape)) for k, p in m.named_parameters()], shape)
        with torch.no_grad():
            for k, p in m.named_parameters():
                p.copy_(params[k])
        x.requires_grad_(True)
        y = m(x)
        gy = draw_gy(y.shape)
        y.backward(gy)
        out = {}
        for k, t in [("y", y.detach()), ("dx", x.grad)] + [("grad." + k, p.grad) for k, p in m.named_parameters()]:
            a = t.numpy().astype(np.float32)
            out["idx." + k], out["sample." + k] = sample(a)
            out["norm." + k] = np.float64(np.linalg.norm(a.astype(np.float64)))
            out["sum." + k] = np.float64(a.astype(np.float64).sum())
        meta = dict(kind="mv", seeded=True, shape=shape, params=[(k, tuple(p.shape)) for k, p in m.named_parameters()],
                    **kw)
        assert names == [k for k, _ in meta["params"]]
        np.savez_compressed(os.path.join(HERE, f"attn_{name}.npz"), meta=np.array(repr(meta)), **out)
        print(name, {k: v.shape for k, v in out.items()})
    for name, kind, kw, shape in cases:
        if only and name not in only:
            continue
        g = torch.Generator().manual_seed(zlib.crc32(name.encode()))
        if kind == "memeff":
            m = MemEffAttention(kw["dim"], kw["num_heads"], qkv_bias=False, proj_bias=True)
        else:
            m = MVAttention(kw["dim"], kw["num_heads"], num_frames=kw["num_frames"], skip_scale=kw["skip_scale"])
        with torch.no_grad():
            for p in m.parameters():
                p.copy_(torch.randn(p.shape, generator=g) * (0.5 / np.sqrt(p.shape[-1]) if p.dim() > 1 else 0.1))
            if kind == "mv":  # non-trivial GroupNorm affine
                m.norm.weight.add_(1.0)
        x = torch.randn(shape, generator=g, requires_grad=True)
        y = m(x)
        gy = torch.randn(y.shape, generator=g)
        y.backward(gy)
        out = {"x": x.detach().numpy(), "gy": gy.numpy(), "y": y.detach().numpy(), "dx": x.grad.numpy()}
        for k, v in m.state_dict().items():
            out["param." + k] = v.numpy()
        for k, p in m.named_parameters():
            out["grad." + k] = p.grad.numpy()
        meta = dict(kind=kind, **kw)
        np.savez_compressed(os.path.join(HERE, f"attn_{name}.npz"), meta=np.array(repr(meta)), **out)
        print(name, {k: v.shape for k, v in out.items() if not k.startswith("param")})


if __name__ == "__main__":
    main()
