#!/bin/bash
# GPU session: the whole -m gpu suite (one process), then the default bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest_exit=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -10
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc2=$?; echo "bench_exit=$rc2"; tail -3 gpurun_out/bench.err
python -c "import json;b=json.load(open('gpurun_out/bench.json'));print(b['value'],b['ms_per_step'],b['kernels']);[print(k,b[k]) for k in ('cfg3_view_sharded','cfg2','cfg4','cfg5','cpu_baseline','roofline')]"
exit $(( rc | rc2 ))
