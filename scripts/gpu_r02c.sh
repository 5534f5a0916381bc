#!/bin/bash
# GPU session: new head / loss tests first, then the full GPU suite, then the bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PYT="python -u -m pytest -v -rA --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_head.py tests/test_loss_gpu.py -m gpu > gpurun_out/new_tests.log 2>&1
rc=$?; echo "new_exit=$rc"; grep -E "FAILED|passed|failed" gpurun_out/new_tests.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 $PYT tests -m gpu --deselect tests/test_head.py --deselect tests/test_loss_gpu.py > gpurun_out/gpu_tests.log 2>&1
rc2=$?; echo "pytest_exit=$rc2"; grep -E "FAILED|passed|failed" gpurun_out/gpu_tests.log | tail -8
[ $rc2 -eq 0 ] || [ $rc2 -eq 1 ] || exit $rc2
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc3=$?; echo "bench_exit=$rc3"; head -c 1200 gpurun_out/bench.json; tail -3 gpurun_out/bench.err
exit $(( rc | rc2 | rc3 ))
