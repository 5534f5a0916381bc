#!/bin/bash
# One GPU session: build, GPU tests, bench, rocprofv3 kernel stats. Every GPU step has its own time limit and
# the chain stops at the first failure (no GPU work after a fault).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
python -m lgm_amd.build > gpurun_out/build.log 2>&1 || { echo "build failed"; exit 1; }
timeout -k 10 600 python -m pytest tests -m gpu -v -rA -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest_exit=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/diag_counters.py > gpurun_out/counters.log 2>&1 || { echo "counters failed"; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-seconds 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench_exit=$rc"; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof.log 2>&1
rc=$?; echo "prof_exit=$rc"; exit $rc
