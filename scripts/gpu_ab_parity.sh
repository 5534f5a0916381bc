#!/bin/bash
# Parity first (the in-tree library: production parity + round-1 render suites + fused loss), then interleaved
# bench rounds over the variant libraries (scripts/gpu_ab.sh). Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_render_parity_gpu.py tests/test_render_gpu.py tests/test_loss_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/ab/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh
