"""Runs only the HIP attention forward (packed qkv, bf16) at one shape, for counter profiles:
python scripts/attn_fwd_only.py B L H D iters [bwd]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lgm_amd.attention import packed_attention  # noqa: E402

B, L, H, D, iters = (int(a) for a in sys.argv[1:6])
bwd = len(sys.argv) > 6 and sys.argv[6] == "bwd"
g = torch.Generator(device="cpu").manual_seed(7)
qkv = torch.randn((B, L, 3, H, D), generator=g).to("cuda", torch.bfloat16)
d_o = torch.randn((B, L, H, D), generator=g).to("cuda", torch.bfloat16)
x = qkv.clone().requires_grad_(bwd)
for _ in range(iters):
    if bwd:
        x.grad = None
        packed_attention(x).backward(d_o)
    else:
        with torch.no_grad():
            packed_attention(x)
torch.cuda.synchronize()
print("done")
