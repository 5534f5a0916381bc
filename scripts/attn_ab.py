"""A/B of attention-kernel variant libraries (lgm_amd/_lib/variants_attn/lib_*.so, built here): per-kernel times of
bench.attention_bench plus a hash of the forward output and the packed gradient, so variants that must be bitwise
equal can be checked in the same run. Each variant runs in its own child process (one library per process)."""
import glob
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, ROOT)
    import torch

    import bench
    from lgm_amd.attention import packed_attention
    dev = torch.device("cuda:0")
    res = bench.attention_bench(dev, steps=20)
    g = torch.Generator(device="cpu").manual_seed(7)
    qkv = torch.randn((8, 4096, 3, 16, 32), generator=g).to(dev, torch.bfloat16).requires_grad_(True)
    d_o = torch.randn((8, 4096, 16, 32), generator=g).to(dev, torch.bfloat16)
    out = packed_attention(qkv)
    out.backward(d_o)
    torch.cuda.synchronize()
    h = lambda t: hashlib.sha1(t.detach().float().cpu().numpy().tobytes()).hexdigest()[:12]  # noqa: E731
    print(json.dumps({"ms": res["ms_per_step"], "kernels": {k: v["avg_us"] for k, v in res["kernels"].items()},
                      "out": h(out), "grad": h(qkv.grad)}))


def main():
    libs = sorted(glob.glob(os.path.join(ROOT, "lgm_amd/_lib/variants_attn/lib_*.so")))
    for rnd in (1, 2):
        for lib in libs:
            env = dict(os.environ, LGM_AMD_LIB=lib)
            p = subprocess.run(["timeout", "-k", "10", "120", sys.executable, __file__, "child"], env=env,
                               capture_output=True, text=True)
            if p.returncode:
                print(os.path.basename(lib), "failed", p.returncode, p.stderr[-2000:])
                sys.exit(p.returncode)
            print(os.path.basename(lib), f"r{rnd}", p.stdout.strip().splitlines()[-1], flush=True)


if __name__ == "__main__":
    child() if sys.argv[1:] == ["child"] else main()
