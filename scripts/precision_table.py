"""Markdown table of the gradient-precision record the GPU suite writes (gpurun_out/grad_precision.json, copied under
profiles/): rel L2 vs the fp64 oracle per parameter group, the fp32 oracle's own error and the test bar.
Usage: python scripts/precision_table.py <grad_precision.json>"""
import json
import sys


def main(path):
    rows = ["| workload | group | GPU vs fp64 | fp32 oracle vs fp64 | bar | GPU vs fp32 oracle |", "|---|---|---|---|---|---|"]
    for t in json.load(open(path)):
        if "groups" not in t:
            continue
        for g, v in t["groups"].items():
            if "gpu" not in v:
                continue
            rows.append(f"| {t['test']} | {g} | {v['gpu']:.2e} | {v['fp32_oracle']:.2e} | {v['bar']:.2e} | "
                        f"{v['gpu_vs_fp32_oracle']:.2e} |")
    print("\n".join(rows))


if __name__ == "__main__":
    main(sys.argv[1])
