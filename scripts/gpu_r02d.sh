#!/bin/bash
# GPU session: render parity (incl. bit-exact tile lists) + head/loss tests with the default library, then the
# interleaved A/B of the variant libraries.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PYT="python -u -m pytest -v -rA --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_render_parity_gpu.py tests/test_render_gpu.py tests/test_head.py tests/test_loss_gpu.py -m gpu > gpurun_out/tests.log 2>&1
rc=$?; echo "tests_exit=$rc"; grep -E "FAILED|passed|failed" gpurun_out/tests.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/gpu_ab.sh
