#!/bin/bash
# (1) the rewritten packed-vs-slot test on the in-tree library, (2) the binning parity tests on the view-loop
# variant library, (3) interleaved A/B timing of the variants. Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_render_parity_gpu.py -x -v --timeout 240 --timeout-method thread -k "exact_count or deterministic" > gpurun_out/check2_tests.log 2>&1
rc=$?; echo "pytest_exit=$rc"; tail -3 gpurun_out/check2_tests.log; [ $rc -eq 0 ] || exit $rc
LGM_AMD_LIB=$PWD/lgm_amd/_lib/variants/lib_vloop.so timeout -k 10 400 python -u -m pytest tests/test_render_parity_gpu.py -x -v --timeout 240 --timeout-method thread -k "integer or headline or cfg3 or production_render" > gpurun_out/check2_vloop.log 2>&1
rc=$?; echo "pytest_vloop_exit=$rc"; tail -3 gpurun_out/check2_vloop.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh > gpurun_out/ab_check2.log 2>&1
rc=$?; cat gpurun_out/ab_check2.log; exit $rc
