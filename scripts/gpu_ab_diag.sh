cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_check.sh tests/test_render_parity_gpu.py tests/test_training_gpu.py || exit $?
bash scripts/gpu_diag_spread.sh 1 || exit $?
