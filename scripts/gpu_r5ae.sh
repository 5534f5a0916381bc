#!/bin/bash
# Round-5 session AE: k_render_fwd pulling the next chunk's records into L2 while the current chunk composites (LDS DMA
# into a junk area; LGM_FWD_PF=1 always, =2 only while under half the tile's pixels are saturated) against none
# (pf0): render GPU tests on pf1 / pf2, then bench.py pool + single scene, two interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5ae
V=$PWD/lgm_amd/_lib/variants
for n in pf1 pf2; do
  LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_render_cases.py tests/test_render_gpu.py tests/test_render_parity_gpu.py -m gpu > gpurun_out/r5ae/t_$n.log 2>&1
  rc=$?; echo "$n tests: $(tail -1 gpurun_out/r5ae/t_$n.log)"; [ $rc -eq 0 ] || exit $rc
done
for round in 1 2; do
  for n in pf0 pf1 pf2; do
    LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cfg4 --no-cfg5 --no-attention --no-cpu-baseline --no-det > gpurun_out/r5ae/b_${n}_r${round}.json 2> gpurun_out/r5ae/b_${n}_r${round}.err || exit $?
    python -c "
import json
b=json.load(open('gpurun_out/r5ae/b_${n}_r${round}.json')); c=b['cfg3_view_sharded']
print('$n r$round pool', b['ms_per_step'], {k: v['avg_us'] for k, v in b['kernels'].items()}, 'cfg3', c['ms_per_step'], {k: v['avg_us'] for k, v in c['kernels'].items()})"
  done
done
