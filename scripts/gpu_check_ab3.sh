#!/bin/bash
# Binning parity tests on the in-tree library (bit-exact radii / K / tile lists, production parity), then the
# interleaved A/B timing of the variant libraries. Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_render_parity_gpu.py -x -v --timeout 240 --timeout-method thread -k "integer or headline or cfg3 or production_render or exact_count" > gpurun_out/check3_tests.log 2>&1
rc=$?; echo "pytest_exit=$rc"; tail -3 gpurun_out/check3_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh > gpurun_out/ab_check3.log 2>&1
rc=$?; cat gpurun_out/ab_check3.log; exit $rc
