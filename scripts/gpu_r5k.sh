#!/bin/bash
# Round-5 session K: k_bin's LDS tile histogram with the bank swizzle (lib_binswz, LGM_BIN_SWZ) vs the same source
# without it (lib_base): output hashes (must match), then bench.py pool + single scene, two interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5k
V=$PWD/lgm_amd/_lib/variants
for n in base binswz; do
  LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 120 python scripts/render_hashes.py > gpurun_out/r5k/hash_$n.json 2>/dev/null || exit $?
  echo "$n hashes $(cat gpurun_out/r5k/hash_$n.json)"
done
for round in 1 2; do
  for n in base binswz; do
    LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cfg4 --no-cfg5 --no-attention --no-cpu-baseline --no-det > gpurun_out/r5k/b_${n}_r${round}.json 2> gpurun_out/r5k/b_${n}_r${round}.err || exit $?
    python -c "
import json
b=json.load(open('gpurun_out/r5k/b_${n}_r${round}.json')); c=b['cfg3_view_sharded']
print('$n r$round pool', b['ms_per_step'], {k: v['avg_us'] for k, v in b['kernels'].items()}, 'cfg3', c['ms_per_step'], {k: v['avg_us'] for k, v in c['kernels'].items()})"
  done
done
