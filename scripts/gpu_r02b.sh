#!/bin/bash
# GPU session: the cfg4 tests (512^2 render, attention shapes), then the bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PYT="python -u -m pytest -v -rA --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_render_parity_gpu.py -m gpu -k "cfg4 or 512" -s > gpurun_out/cfg4_tests.log 2>&1
rc=$?; echo "cfg4_exit=$rc"; tail -4 gpurun_out/cfg4_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 $PYT tests/test_attention.py -m gpu > gpurun_out/attn_tests.log 2>&1
rc2=$?; echo "attn_exit=$rc2"; tail -4 gpurun_out/attn_tests.log
[ $rc2 -eq 0 ] || [ $rc2 -eq 1 ] || exit $rc2
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc3=$?; echo "bench_exit=$rc3"; tail -c 1500 gpurun_out/bench.json; tail -5 gpurun_out/bench.err
exit $(( rc | rc2 | rc3 ))
