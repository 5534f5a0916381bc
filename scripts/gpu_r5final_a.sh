#!/bin/bash
# Round-5 end, part A: the whole -m gpu suite in one process, then smoke().
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/final
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1
rc=$?; echo "pytest_exit=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/final/gpu_tests.log | tail -10
cp gpurun_out/grad_precision.json gpurun_out/final/ 2>/dev/null
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1
rs=$?; echo "smoke_exit=$rs"; tail -2 gpurun_out/final/smoke.log; exit $rs
