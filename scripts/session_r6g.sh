cd $GRAFT_REPO_ROOT && OUT=gpurun_out/r6g bash scripts/gpu_run.sh "tests=tests/test_wgrad.py" || exit $?
mkdir -p gpurun_out/r6g/wg
for r in 1 2; do for v in s256 s512 s1024; do
  LGM_AMD_LIB=$GRAFT_REPO_ROOT/lgm_amd/_lib/variants/lib_$v.so timeout -k 10 120 python scripts/bench_wgrad.py > gpurun_out/r6g/wg/${v}_r$r.jsonl 2>&1 || exit $?
  echo "$v r$r"; cat gpurun_out/r6g/wg/${v}_r$r.jsonl
done; done
