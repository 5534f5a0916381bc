#!/bin/bash
# Round-end session at HEAD: the GPU suite, smoke, rocprofv3 kernel stats + PMC passes (scripts/gpu_session.sh),
# then the default bench line twice unprofiled (as the driver runs it).
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_session.sh || exit $?
for r in 1 2; do
  echo "== bench $r $(date +%s)"
  timeout -k 10 400 python bench.py > gpurun_out/bench_plain$r.json 2> gpurun_out/bench_plain$r.err || exit $?
  python -c "import json;b=json.load(open('gpurun_out/bench_plain$r.json'));c=b['cfg3_view_sharded'];print(b['value'], b['ms_per_step'], b['step_spread'], b['kernels'], 'cfg3', c['ms_per_step'], c['step_spread'], 'cfg2', b['cfg2']['ms_per_step'], 'cfg5', b['cfg5']['render_side_ms'], 'cfg4', b['cfg4']['attention_ms'], b['cfg4']['render_ms'], 'attn', b['attention']['tflops'], b['attention']['kernels'])"
done
