cd $GRAFT_REPO_ROOT && OUT=gpurun_out/r6h bash scripts/gpu_run.sh "tests=tests/test_wgrad.py tests/test_attention.py -k mvattention" || exit $?
timeout -k 10 120 python scripts/bench_wgrad.py > gpurun_out/r6h/bench_wgrad.jsonl 2>&1 || exit $?
cat gpurun_out/r6h/bench_wgrad.jsonl
OUT=gpurun_out/r6h bash scripts/gpu_run.sh "benchargs=--only-attn --steps 10"
