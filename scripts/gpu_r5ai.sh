#!/bin/bash
# Round-5 session AI: as AH, plus pl2 (LGM_PRE_LDS=2: the Gaussian, its first view and its scene partials loaded
# before the matrix staging) against pl1 and HEAD (pl0): hashes, render tests on pl2, pool + single scene.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5ai
V=$PWD/lgm_amd/_lib/variants
for n in pl0 pl1 pl2; do
  LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 120 python scripts/render_hashes.py > gpurun_out/r5ai/hash_$n.json 2>/dev/null || exit $?
  echo "$n hashes $(cat gpurun_out/r5ai/hash_$n.json)"
done
LGM_AMD_LIB=$V/lib_pl2.so timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_render_cases.py tests/test_render_gpu.py tests/test_render_parity_gpu.py -m gpu > gpurun_out/r5ai/t_pl2.log 2>&1
rc=$?; echo "pl2 tests: $(tail -1 gpurun_out/r5ai/t_pl2.log)"; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for n in pl0 pl1 pl2; do
    LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cfg4 --no-cfg5 --no-attention --no-cpu-baseline --no-det > gpurun_out/r5ai/b_${n}_r${round}.json 2> gpurun_out/r5ai/b_${n}_r${round}.err || exit $?
    python -c "
import json
b=json.load(open('gpurun_out/r5ai/b_${n}_r${round}.json')); c=b['cfg3_view_sharded']
print('$n r$round pool', b['ms_per_step'], {k: v['avg_us'] for k, v in b['kernels'].items()}, 'cfg3', c['ms_per_step'], {k: v['avg_us'] for k, v in c['kernels'].items()})"
  done
done
