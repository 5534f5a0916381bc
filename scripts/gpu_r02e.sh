#!/bin/bash
# GPU session: render tests, then the default bench line and per-grid kernel stats of a profiled bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
PYT="python -u -m pytest -v -rA --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_render_parity_gpu.py tests/test_render_gpu.py tests/test_loss_gpu.py -m gpu > gpurun_out/tests.log 2>&1
rc=$?; echo "tests_exit=$rc"; grep -E "FAILED|passed|failed" gpurun_out/tests.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err
rc2=$?; echo "bench_exit=$rc2"; python scripts/kernel_stats_by_grid.py gpurun_out/prof/run_kernel_trace.csv > gpurun_out/prof/kernel_stats_by_grid.txt; head -20 gpurun_out/prof/kernel_stats_by_grid.txt
python -c "import json;b=json.load(open('gpurun_out/prof/bench.json'));print(b['value'],b['ms_per_step'],b['cfg3_view_sharded'],b['cfg4'],b['cfg2'])"
exit $(( rc | rc2 ))
