"""Print the key numbers of gpurun_out/bench.json and gpurun_out/prof/run_kernel_stats.csv."""
import csv
import json
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
b = json.load(open(f"{root}/bench.json"))
c = b["config"]
print(f"value {b['value']} Mpix/s  ms/step {b['ms_per_step']}  K_ref {c.get('pairs_K_reference')} binned {c.get('pairs_binned')}")
print("roofline", b["roofline"])
print("step", b["step_roofline"])
if "cpu_baseline" in b:
    print("cpu", b["cpu_baseline"]["value"], b["cpu_baseline"]["unit"], "cores", b["cpu_baseline"]["cores"])
for k, v in b["kernels"].items():
    print(f"  {k:16s} {v['avg_us']:9.2f} us")
try:
    rows = list(csv.DictReader(open(f"{root}/prof/run_kernel_stats.csv")))
    print("rocprof:")
    for r in rows[:8]:
        n = r["Name"].split("(")[0].split("::")[-1][:40]
        print(f"  {n:40s} calls={r['Calls']:>4} avg_us={float(r['AverageNs']) / 1e3:9.2f} pct={float(r['Percentage']):6.2f}")
except FileNotFoundError:
    pass
