#!/bin/bash
# Counter passes over the attention kernels alone (scripts/attn_fwd_only.py), one rocprofv3 run per pass.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc_attn
export TMPDIR=/tmp
SHAPE=${SHAPE:-"1 9600 16 32 5"}
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $line -d gpurun_out/pmc_attn/p$i -o run --output-format csv -- python scripts/attn_fwd_only.py $SHAPE $MODE > gpurun_out/pmc_attn/p$i.log 2>&1
  rc=$?; echo "pass $i ($line) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done < scripts/pmc_passes_attn.txt
