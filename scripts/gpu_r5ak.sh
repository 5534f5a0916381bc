#!/bin/bash
# Round-5 session AK: the compositing kernels' first list ids loaded before the list length in slot mode
# (LGM_SPEC_IDS=1: lib_sp1) against HEAD (lib_sp0): hashes (must match), render GPU tests on sp1, then bench.py
# pool + single scene, two interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5ak
V=$PWD/lgm_amd/_lib/variants
for n in sp0 sp1; do
  LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 120 python scripts/render_hashes.py > gpurun_out/r5ak/hash_$n.json 2>/dev/null || exit $?
  echo "$n hashes $(cat gpurun_out/r5ak/hash_$n.json)"
done
LGM_AMD_LIB=$V/lib_sp1.so timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_render_cases.py tests/test_render_gpu.py tests/test_render_parity_gpu.py -m gpu > gpurun_out/r5ak/t_sp1.log 2>&1
rc=$?; echo "sp1 tests: $(tail -1 gpurun_out/r5ak/t_sp1.log)"; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for n in sp0 sp1; do
    LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cfg4 --no-cfg5 --no-attention --no-cpu-baseline --no-det > gpurun_out/r5ak/b_${n}_r${round}.json 2> gpurun_out/r5ak/b_${n}_r${round}.err || exit $?
    python -c "
import json
b=json.load(open('gpurun_out/r5ak/b_${n}_r${round}.json')); c=b['cfg3_view_sharded']
print('$n r$round pool', b['ms_per_step'], {k: v['avg_us'] for k, v in b['kernels'].items()}, 'cfg3', c['ms_per_step'], {k: v['avg_us'] for k, v in c['kernels'].items()})"
  done
done
