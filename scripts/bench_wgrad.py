"""k_wgrad / k_wgrad_reduce per shape (HIP-event kernel times, lgm_amd's KernelProfiler) for the library in
LGM_AMD_LIB: the bench's MVAttention level (qkv: K 32768 x 1536 x 512; proj: 512 x 512 with its bias) and cfg4's
L = 9600 level. Prints one JSON line per shape."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from lgm_amd import _native  # noqa: E402

dev = torch.device("cuda:0")
L = _native.lib()
for K, M, N, want_db in [(32768, 1536, 512, False), (32768, 512, 512, True), (32768, 512, 512, False),
                         (9600, 1536, 512, False), (9600, 512, 512, True)]:
    g = torch.Generator().manual_seed(1)
    dy = torch.randn((K, M), generator=g).to(dev, torch.bfloat16)
    x = torch.randn((K, N), generator=g).to(dev, torch.bfloat16)
    dw = torch.empty((M, N), device=dev)
    db = torch.empty((M,), device=dev) if want_db else None
    ws_bytes = L.lgm_linear_wgrad_workspace_size(K, M, N, int(want_db))
    ws = torch.empty(ws_bytes, device=dev, dtype=torch.uint8)

    def call():
        _native.check(L.lgm_linear_wgrad(1, K, M, N, _native.ptr(dy), M, _native.ptr(x), N, _native.ptr(dw),
                                         _native.ptr(db), _native.ptr(ws), ws_bytes, _native.stream_of(dev),
                                         _native.diag()), "lgm_linear_wgrad")
    for _ in range(5):
        call()
    torch.cuda.synchronize()
    prof = _native.KernelProfiler()
    with prof:
        for _ in range(20):
            call()
        torch.cuda.synchronize()
    s = prof.summary()
    prof.close()
    us = {k: round(1e3 * v / n, 2) for k, (n, v) in s.items()}
    tf = 2.0 * K * M * N / (us["k_wgrad"] * 1e-6) / 1e12
    print(json.dumps({"K": K, "M": M, "N": N, "db": want_db, "us": us, "wgrad_tflops": round(tf, 1),
                      "ws_MB": round(ws_bytes / 1e6, 1)}), flush=True)
