#!/bin/bash
# SQ counter passes (scripts/pmc_passes.txt lines 1-2) for every variant library: gpurun_out/pmc_ab/<lib>/p<i>.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for lib in lgm_amd/_lib/variants/lib_*.so; do
  n=$(basename $lib .so)
  i=0
  head -2 scripts/pmc_passes.txt | while read -r line; do
    i=$((i+1))
    mkdir -p gpurun_out/pmc_ab/$n
    LGM_AMD_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc $line -d gpurun_out/pmc_ab/$n/p$i -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-attention > gpurun_out/pmc_ab/$n/p$i.log 2>&1
    rc=$?; echo "$n pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done || exit 1
  python scripts/pmc_summary.py gpurun_out/pmc_ab/$n > gpurun_out/pmc_ab/$n/summary.txt
done
