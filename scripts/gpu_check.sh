#!/bin/bash
# Quick GPU check: selected pytest files (args: pytest node ids / files, default the whole -m gpu suite), then the
# interleaved A/B of variant libraries if any were built (scripts/gpu_ab.sh). Stops at the first hard failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ARGS=("$@"); [ ${#ARGS[@]} -eq 0 ] && ARGS=(tests)
timeout -k 10 900 python -u -m pytest "${ARGS[@]}" -m gpu -v -rA --timeout 300 --timeout-method thread > gpurun_out/gpu_check.log 2>&1
rc=$?; echo "pytest_exit=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_check.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
if ls lgm_amd/_lib/variants/lib_*.so > /dev/null 2>&1; then bash scripts/gpu_ab.sh || exit $?; fi
exit $rc
