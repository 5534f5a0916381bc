#!/bin/bash
# Round-5 session Y (probe): k_render_bwd with 4 / 8 extra independent FMAs per (entry, pixel) on dummy chains
# (lib_pad4 / lib_pad8, LGM_BWD_PAD_VALU) against the same source without them (lib_base): does the backward's time
# follow its VALU count (~34 per (entry, pixel))? bench.py pool + single scene, two interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5y
V=$PWD/lgm_amd/_lib/variants
for round in 1 2; do
  for n in base pad4 pad8; do
    LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cfg4 --no-cfg5 --no-attention --no-cpu-baseline --no-det > gpurun_out/r5y/b_${n}_r${round}.json 2> gpurun_out/r5y/b_${n}_r${round}.err || exit $?
    python -c "
import json
b=json.load(open('gpurun_out/r5y/b_${n}_r${round}.json')); c=b['cfg3_view_sharded']
print('$n r$round pool', b['ms_per_step'], {k: v['avg_us'] for k, v in b['kernels'].items()}, 'cfg3', c['ms_per_step'], {k: v['avg_us'] for k, v in c['kernels'].items()})"
  done
done
