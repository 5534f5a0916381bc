set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python -m lgm_amd.build > gpurun_out/build2.log 2>&1
timeout -k 10 600 python -m pytest tests -m gpu -v -rA > gpurun_out/gpu2.log 2>&1
echo "pytest_exit=$?" >> gpurun_out/gpu2.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-seconds 5 > gpurun_out/bench2.json 2> gpurun_out/bench2.err
echo "bench_exit=$?"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof2.log 2>&1
echo "prof_exit=$?"
