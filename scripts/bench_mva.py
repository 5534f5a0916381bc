"""bench.py's MVAttention level alone (one block fwd+bwd, fused layout vs torch ops): one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import bench
    print(json.dumps(bench.mva_level_bench(torch.device("cuda", 0), steps=20)))


if __name__ == "__main__":
    main()
