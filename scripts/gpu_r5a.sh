#!/bin/bash
# Round-5 session A: the pool stall of BENCH_r04. The driver's command with the round-4 warm-up (per-step stamps),
# then bench.py with the new warm-up (first call out of the rate estimate), both as the driver runs them.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5a
timeout -k 10 300 python scripts/diag_warmup.py --steps 20 --warmup 5 --only-pool > gpurun_out/r5a/legacy.json 2> gpurun_out/r5a/legacy.err || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5a/bench.json 2> gpurun_out/r5a/bench.err || exit $?
timeout -k 10 300 python scripts/diag_warmup.py --steps 20 --warmup 5 --only-pool > gpurun_out/r5a/legacy2.json 2> gpurun_out/r5a/legacy2.err || exit $?
for f in legacy bench legacy2; do
python -c "
import json
b=json.load(open('gpurun_out/r5a/$f.json'))
t=b['timed_loop']
print('$f', b['ms_per_step'], b['step_spread'], 'loop', t['loop_ms'], 'gpu_sum', t['gpu_sum_ms'], 'tail', t['tail_ms'])
print('  gpu', t['gpu_ms'])
print('  host', t['host_ms'])
c=b.get('cfg3_view_sharded')
if c: print('  cfg3', c['ms_per_step'], c['step_spread'], c['timed_loop']['gpu_ms'])
"
done
grep legacy gpurun_out/r5a/*.err
