#!/bin/bash
# Round-5 session AQ: the forward of a one-round grid capped at 4 / 5 workgroups per CU by unused dynamic LDS
# (LGM_FWD_CAP=4 / 5: lib_cap4 / lib_cap5) against HEAD (lib_cap0): hashes, render tests on cap5, then bench.py
# pool + single scene, two interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5aq
V=$PWD/lgm_amd/_lib/variants
for n in cap0 cap4 cap5; do
  LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 120 python scripts/render_hashes.py > gpurun_out/r5aq/hash_$n.json 2>/dev/null || exit $?
  echo "$n hashes $(cat gpurun_out/r5aq/hash_$n.json)"
done
LGM_AMD_LIB=$V/lib_cap5.so timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_render_cases.py tests/test_render_gpu.py tests/test_render_parity_gpu.py -m gpu > gpurun_out/r5aq/t_cap5.log 2>&1
rc=$?; echo "cap5 tests: $(tail -1 gpurun_out/r5aq/t_cap5.log)"; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for n in cap0 cap4 cap5; do
    LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cfg4 --no-cfg5 --no-attention --no-cpu-baseline --no-det > gpurun_out/r5aq/b_${n}_r${round}.json 2> gpurun_out/r5aq/b_${n}_r${round}.err || exit $?
    python -c "
import json
b=json.load(open('gpurun_out/r5aq/b_${n}_r${round}.json')); c=b['cfg3_view_sharded']
print('$n r$round pool', b['ms_per_step'], {k: v['avg_us'] for k, v in b['kernels'].items()}, 'cfg3', c['ms_per_step'], {k: v['avg_us'] for k, v in c['kernels'].items()})"
  done
done
