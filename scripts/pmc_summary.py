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

if "--json" in sys.argv:  # per-dispatch HBM bytes for bench.py's roofline.traffic (MI355X_MICROARCH.md §HBM)
    import json
    import subprocess
    out = {}
    for name, cs in agg.items():
        m = {cn: sum(v) / len(v) for cn, v in cs.items()}
        rec = {}
        if "FETCH_SIZE" in m:
            rec["hbm_read_bytes"] = 2 * m["FETCH_SIZE"] * 1024  # KiB, x2: gfx950 tallies 128-B reads at 64 B
        if "WRITE_SIZE" in m:
            rec["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVES"):
            if k in m:
                rec[k] = m[k]
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            if "SQ_WAIT_ANY" in m:
                rec["wait_frac"] = round(m["SQ_WAIT_ANY"] / wc, 4)
            if "SQ_ACTIVE_INST_VALU" in m:
                rec["valu_busy_frac"] = round(m["SQ_ACTIVE_INST_VALU"] / wc, 4)
        if m.get("SQ_LDS_IDX_ACTIVE"):
            rec["lds_bank_conflict_frac"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0.0) / m["SQ_LDS_IDX_ACTIVE"], 4)
        out[name.split("<")[0]] = rec
    import os
    rev = os.environ.get("PMC_COMMIT", "")
    if not rev:
        try:
            rev = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True).stdout.strip()
        except OSError:
            rev = ""
    out["_meta"] = {"source": root, "commit": rev,
                    "workload": os.environ.get("PMC_WORKLOAD", "bench.py --only-pool (8-scene pool, cfg3 scenes)"),
                    "command": "rocprofv3 --kernel-trace --pmc <pass> -- python bench.py --steps 3 --warmup 2 "
                               "--only-pool --no-cpu-baseline"}
    path = sys.argv[sys.argv.index("--json") + 1]
    json.dump(out, open(path, "w"), indent=1)
    print("wrote", path)
