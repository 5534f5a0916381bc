#!/bin/bash
# Round-5 session T: the chunk commit's quadrant test with 1-ulp reciprocals (lib_rcp, LGM_COMMIT_RCP) vs the same
# source with IEEE divisions (lib_base): output hashes (must match), then bench.py pool + single scene, two rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5t
V=$PWD/lgm_amd/_lib/variants
for n in base rcp; do
  LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 120 python scripts/render_hashes.py > gpurun_out/r5t/hash_$n.json 2>/dev/null || exit $?
  echo "$n hashes $(cat gpurun_out/r5t/hash_$n.json)"
done
for round in 1 2; do
  for n in base rcp; do
    LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cfg4 --no-cfg5 --no-attention --no-cpu-baseline --no-det > gpurun_out/r5t/b_${n}_r${round}.json 2> gpurun_out/r5t/b_${n}_r${round}.err || exit $?
    python -c "
import json
b=json.load(open('gpurun_out/r5t/b_${n}_r${round}.json')); c=b['cfg3_view_sharded']
print('$n r$round pool', b['ms_per_step'], {k: v['avg_us'] for k, v in b['kernels'].items()}, 'cfg3', c['ms_per_step'], {k: v['avg_us'] for k, v in c['kernels'].items()})"
  done
done
