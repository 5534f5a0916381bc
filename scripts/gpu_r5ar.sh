#!/bin/bash
# Round-5 session AR: k_head_bwd with its dL/dgaussians row loads all in flight (lib_h1) against HEAD (lib_h0): head
# GPU tests on h1, then rocprofv3 kernel stats of the cfg5 line per library (k_head_bwd's average).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5ar
V=$PWD/lgm_amd/_lib/variants
LGM_AMD_LIB=$V/lib_h1.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_head.py tests/test_training_gpu.py -m gpu > gpurun_out/r5ar/t_h1.log 2>&1
rc=$?; echo "h1 tests: $(tail -1 gpurun_out/r5ar/t_h1.log)"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for n in h0 h1 h0 h1; do
  LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r5ar/prof_$n -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cfg4 --no-attention --no-cpu-baseline --no-det > $GRAFT_REPO_ROOT/gpurun_out/r5ar/b_$n.log 2>&1 || exit $?
  f=$(find $GRAFT_REPO_ROOT/gpurun_out/r5ar/prof_$n -name "*kernel_stats.csv" | head -1)
  echo "$n $(grep -h k_head_bwd $f | cut -d, -f1-5)"
done
