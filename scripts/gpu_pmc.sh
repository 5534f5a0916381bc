#!/bin/bash
# PMC passes (one rocprofv3 run per pass; counters only with --kernel-trace, no other trace domains).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
python -m lgm_amd.build > gpurun_out/build.log 2>&1 || { echo "build failed"; exit 1; }
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $line -d gpurun_out/pmc/p$i -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-attention > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($line) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done < scripts/pmc_passes.txt
