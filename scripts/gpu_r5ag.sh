#!/bin/bash
# Round-5 session AG: tiles of each XCD group in runs of 32 rotated by 5 per run (xcd_item_rot) so a CU's first-round
# tiles spread over columns: LGM_TILE_ROT=1 forward, =3 forward + backward heads, against raster order (rot0):
# render GPU tests on rot1 / rot3, scripts/diag_cu.py per library, then bench.py pool + single scene, two rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5ag
V=$PWD/lgm_amd/_lib/variants
for n in rot1 rot3; do
  LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_render_cases.py tests/test_render_gpu.py tests/test_render_parity_gpu.py -m gpu > gpurun_out/r5ag/t_$n.log 2>&1
  rc=$?; echo "$n tests: $(tail -1 gpurun_out/r5ag/t_$n.log)"; [ $rc -eq 0 ] || exit $rc
done
for n in rot0 rot1 rot3; do
  LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 240 python scripts/diag_cu.py > gpurun_out/r5ag/cu_$n.json 2> gpurun_out/r5ag/cu_$n.err || exit $?
done
for round in 1 2; do
  for n in rot0 rot1 rot3; do
    LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cfg4 --no-cfg5 --no-attention --no-cpu-baseline --no-det > gpurun_out/r5ag/b_${n}_r${round}.json 2> gpurun_out/r5ag/b_${n}_r${round}.err || exit $?
    python -c "
import json
b=json.load(open('gpurun_out/r5ag/b_${n}_r${round}.json')); c=b['cfg3_view_sharded']
print('$n r$round pool', b['ms_per_step'], {k: v['avg_us'] for k, v in b['kernels'].items()}, 'cfg3', c['ms_per_step'], {k: v['avg_us'] for k, v in c['kernels'].items()})"
  done
done
