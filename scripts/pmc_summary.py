"""Aggregate rocprofv3 counter CSVs (gpurun_out/pmc/p*/run_counter_collection.csv): per kernel, mean per dispatch."""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_[a-z_]+(?:<[^>]*>)?)", r["Kernel_Name"])
        if "lgm" not in r["Kernel_Name"] or not m:
            continue
        name = m.group(1)
        per[(name, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (name, did, cn), v in per.items():
        agg[name][cn].append(v)
for name, cs in agg.items():
    print(name)
    m = {cn: sum(v) / len(v) for cn, v in cs.items()}
    for cn in sorted(m):
        print(f"   {cn:28s} {m[cn]:.4g}")
    if "SQ_WAVE_CYCLES" in m:
        wc = m["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
            if k in m:
                print(f"   {k + '/WAVE_CYCLES':40s} {m[k] / wc:.3f}")
    if "FETCH_SIZE" in m:
        print(f"   HBM read (2 x FETCH_SIZE, gfx950 correction) MB {2 * m['FETCH_SIZE'] / 1e3:.2f}")
    if "WRITE_SIZE" in m:
        print(f"   HBM write MB {m['WRITE_SIZE'] / 1e3:.2f}")
