"""bench.py's MVAttention level, fused path only (C = 512, 32x32 x 4 views, 16 heads, 8 objects, fwd+bwd, bf16
autocast), STEPS steps after a warm-up: for rocprofv3 kernel traces of everything one training step of the block
launches (library GEMMs and torch's elementwise kernels included). python scripts/probe_mva_train.py [STEPS]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from lgm_amd.attention import MVAttention  # noqa: E402

dev = torch.device("cuda:0")
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B, F, C, HH, WW = 8, 4, 512, 32, 32
torch.manual_seed(3)
m = MVAttention(C, 16, num_frames=F, skip_scale=0.5 ** 0.5).to(dev)
x = (torch.randn(B * F, C, HH, WW, device=dev) * 2 + 0.3).requires_grad_(True)
gy = torch.randn(B * F, C, HH, WW, device=dev)


def step():
    x.grad = None
    m.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    y.backward(gy)


for _ in range(5):
    step()
torch.cuda.synchronize()
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
st.record()
for _ in range(steps):
    step()
en.record()
torch.cuda.synchronize()
print(f"ms_per_step {st.elapsed_time(en) / steps:.4f}")
