#!/bin/bash
# Round-4 session V: the default bench line (as the driver runs it, unprofiled) twice with the time-floored warmup
# (dist.warm_up), and the multi-process GPU tests.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2; do
  echo "== bench $r $(date +%s)"
  timeout -k 10 400 python bench.py > gpurun_out/bench_plain$r.json 2> gpurun_out/bench_plain$r.err || exit $?
  python -c "import json;b=json.load(open('gpurun_out/bench_plain$r.json'));c=b['cfg3_view_sharded'];print(b['value'], b['ms_per_step'], b['step_spread'], 'cfg3', c['ms_per_step'], c['step_spread'], 'cfg2', b['cfg2']['ms_per_step'], 'cfg5', b['cfg5']['render_side_ms'], 'attn', b['attention']['tflops'], b['attention']['kernels'])"
done
echo "== dist tests $(date +%s)"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_dist_gpu.py > gpurun_out/t_dist.log 2>&1
rc=$?; tail -2 gpurun_out/t_dist.log; exit $rc
