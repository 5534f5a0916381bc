#!/bin/bash
# Round-5 session E: timing only, HEAD vs the wave-flush backward (lib_wflush), bench.py pool + single scene, two
# interleaved rounds (its 512^2 needle precision is being fixed separately).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5e
V=$PWD/lgm_amd/_lib/variants
for round in 1 2; do
  for n in head wflush; do
    if [ $n = head ]; then unset LGM_AMD_LIB; else export LGM_AMD_LIB=$V/lib_$n.so; fi
    timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cfg4 --no-cfg5 --no-attention --no-cpu-baseline --no-det > gpurun_out/r5e/b_${n}_r${round}.json 2> gpurun_out/r5e/b_${n}_r${round}.err || exit $?
    python -c "
import json
b=json.load(open('gpurun_out/r5e/b_${n}_r${round}.json')); c=b['cfg3_view_sharded']
print('$n r$round pool', b['ms_per_step'], b['step_spread']['median_ms'], {k: v['avg_us'] for k, v in b['kernels'].items()}, 'cfg3', c['ms_per_step'], c['step_spread']['median_ms'], {k: v['avg_us'] for k, v in c['kernels'].items()})"
  done
done
