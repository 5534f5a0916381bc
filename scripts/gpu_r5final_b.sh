#!/bin/bash
# Round-5 end, part B: rocprofv3 kernel stats of the default bench + the PMC passes of the headline workload
# (scripts/gpu_prof.sh), then bench.py unprofiled: twice with the defaults, once with the driver's arguments.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/final
PMC_COMMIT=${PMC_COMMIT:-unknown} bash scripts/gpu_prof.sh || exit $?
python scripts/kernel_stats_by_grid.py gpurun_out/prof/run_kernel_trace.csv > gpurun_out/prof/kernel_stats_by_grid.txt
for r in 1 2; do
  timeout -k 10 400 python bench.py > gpurun_out/final/bench_plain$r.json 2> gpurun_out/final/bench_plain$r.err || exit $?
done
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/bench_driver_args.json 2> gpurun_out/final/bench_driver_args.err || exit $?
for f in bench_plain1 bench_plain2 bench_driver_args; do
python -c "
import json
b=json.load(open('gpurun_out/final/$f.json')); c=b['cfg3_view_sharded']
print('$f', b['value'], b['ms_per_step'], b['step_spread'], {k: v['avg_us'] for k, v in b['kernels'].items()}, 'cfg3', c['ms_per_step'], c['step_spread'], 'attn', b['attention']['tflops'], 'mva', b.get('mva_level'), 'cfg4', b['cfg4']['attention_ms'], b['cfg4']['attention_core_tflops'], 'cfg5', b['cfg5']['render_side_ms'])"
done
