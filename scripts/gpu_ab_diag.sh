#!/bin/bash
# Selected GPU tests + the interleaved A/B of variant libraries (scripts/gpu_check.sh), then the float-spread
# diagnosis of the default library and of each variant (scripts/gpu_diag_spread.sh; $1 float runs, default 1).
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_check.sh tests/test_render_parity_gpu.py tests/test_training_gpu.py || exit $?
bash scripts/gpu_diag_spread.sh ${1:-1} || exit $?
