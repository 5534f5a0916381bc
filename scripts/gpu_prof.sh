#!/bin/bash
# Profiles of the current tree: rocprofv3 kernel-trace stats of the default bench, then the PMC passes of the
# headline workload (one rocprofv3 run per pass, counters only with --kernel-trace), summarised to JSON.
# Usage: PMC_COMMIT=<sha> bash scripts/gpu_prof.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof gpurun_out/pmc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err
rc=$?; echo "stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $line -d gpurun_out/pmc/p$i -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --only-pool --no-cpu-baseline > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($line) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done < scripts/pmc_passes.txt
python scripts/pmc_summary.py gpurun_out/pmc --json gpurun_out/pmc_latest.json > gpurun_out/pmc_summary.txt
echo "summary rc=$?"
