#!/bin/bash
# GPU session at HEAD: the whole -m gpu suite (one process), smoke(), then rocprofv3 kernel stats of the default
# bench and the PMC passes of the headline workload (scripts/gpu_prof.sh). Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest_exit=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -10
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
rs=$?; echo "smoke_exit=$rs"; tail -2 gpurun_out/smoke.log; [ $rs -eq 0 ] || exit $rs
bash scripts/gpu_prof.sh || exit $?
python scripts/kernel_stats_by_grid.py gpurun_out/prof/run_kernel_trace.csv > gpurun_out/prof/kernel_stats_by_grid.txt
python -c "import json;b=json.load(open('gpurun_out/prof/bench.json'));print(b['value'],b['ms_per_step'],b['kernels']);[print(k,b[k]) for k in ('cfg3_view_sharded','cfg2','cfg4','cfg5','cpu_baseline','roofline')]"
exit $rc
