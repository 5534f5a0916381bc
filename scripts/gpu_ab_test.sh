#!/bin/bash
# Parity-gated A/B: for every variant library, run the GPU render tests against it, then interleaved bench rounds
# (scripts/gpu_ab.sh). Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
for lib in lgm_amd/_lib/variants/lib_*.so; do
  n=$(basename $lib .so)
  LGM_AMD_LIB=$PWD/$lib timeout -k 10 300 python -m pytest tests/test_render_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/${n}_tests.log 2>&1
  rc=$?; echo "$n tests rc=$rc $(tail -1 gpurun_out/ab/${n}_tests.log)"; [ $rc -eq 0 ] || exit $rc
done
bash scripts/gpu_ab.sh
