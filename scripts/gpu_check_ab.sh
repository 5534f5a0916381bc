#!/bin/bash
# Parity tests of the in-tree library that touch the changed kernels, then the interleaved A/B timing of the
# variant libraries (scripts/gpu_ab.sh). Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_render_parity_gpu.py tests/test_render_gpu.py -x -v --timeout 300 --timeout-method thread -k "${LGM_TEST_K:-integer or headline or cfg3 or ties}" > gpurun_out/check_tests.log 2>&1
rc=$?; echo "pytest_exit=$rc"; tail -3 gpurun_out/check_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh > gpurun_out/ab_check.log 2>&1
rc=$?; cat gpurun_out/ab_check.log; exit $rc
