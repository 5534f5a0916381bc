"""Per-(kernel, grid) durations from a rocprofv3 kernel trace (run_kernel_trace.csv): bench.py launches the render
kernels at several sizes (the 8-scene pool, cfg3, cfg2, cfg4), so rocprofv3's per-name averages mix workloads.
Usage: python scripts/kernel_stats_by_grid.py <run_kernel_trace.csv> [> summary.txt]"""
import collections
import csv
import re
import sys

rows = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"]
    m = re.search(r"(k_[a-z_0-9]+(?:<[^>]*>)?)", name)
    short = m.group(1) if m and "lgm" in name else name[:60]
    grid = (int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), int(r["Grid_Size_Y"]))
    rows[(short, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(f"{'kernel':34s} {'grid (wg x, y)':>16s} {'calls':>6s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s} {'total_ms':>9s}")
for (k, g), v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
    if sum(v) < 100:  # < 0.1 ms in total
        continue
    print(f"{k:34s} {str(g):>16s} {len(v):6d} {sum(v) / len(v):9.2f} {min(v):9.2f} {max(v):9.2f} {sum(v) / 1e3:9.3f}")
