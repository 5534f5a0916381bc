#!/bin/bash
# Round-2 GPU session: new parity tests first, then the full GPU suite, then the default bench line.
# Every GPU step has its own time limit; the chain stops at the first failure (no GPU work after a fault).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PYT="python -u -m pytest -v -rA --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_render_parity_gpu.py -m gpu -s > gpurun_out/parity.log 2>&1
rc=$?; echo "parity_exit=$rc"; tail -5 gpurun_out/parity.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ "${ONLY_PARITY:-0}" = 1 ] && exit $rc
timeout -k 10 900 $PYT tests -m gpu --deselect tests/test_render_parity_gpu.py > gpurun_out/gpu_tests.log 2>&1
rc2=$?; echo "pytest_exit=$rc2"; tail -3 gpurun_out/gpu_tests.log
[ $rc2 -eq 0 ] || [ $rc2 -eq 1 ] || exit $rc2
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc3=$?; echo "bench_exit=$rc3"; tail -c 3000 gpurun_out/bench.json; tail -5 gpurun_out/bench.err
exit $(( rc | rc2 | rc3 ))
