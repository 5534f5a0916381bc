"""Precision record of the 16-bit attention kernels: relative L2 of o, dq, dk, dv against the fp64 result of the same
rounded inputs (tests/test_attention.py's seeded inputs), at LGM's D = 32 bench level (L 4096, 16 heads) and cfg4's
L 9600 level. One JSON line per (dtype, shape). Used to compare kernel variants (LGM_AMD_LIB) on the GPU."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

import torch  # noqa: E402

from tests.attn_precision import errors  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    for dtype in (torch.bfloat16, torch.float16):
        for shape in ((1, 4096, 16, 32), (1, 9600, 16, 32), (1, 2400, 16, 64)):
            print(json.dumps({"dtype": str(dtype).split(".")[-1], "shape": shape, **errors(dev, shape, dtype)}),
                  flush=True)
