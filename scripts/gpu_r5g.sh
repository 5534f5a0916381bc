#!/bin/bash
# Round-5 session G: what the backward's gradient flush costs. Timing only: HEAD, no flush at all (noflush, wrong
# gradients), atomics from waves 1-3 only (f123: the stager wave's DMA wait no longer waits for atomics); the f123
# render tests; bench.py pool + single scene, two interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5g
V=$PWD/lgm_amd/_lib/variants
LGM_AMD_LIB=$V/lib_f123.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_render_gpu.py -m gpu > gpurun_out/r5g/t_f123.log 2>&1
rc=$?; tail -1 gpurun_out/r5g/t_f123.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for n in head noflush f123; do
    if [ $n = head ]; then unset LGM_AMD_LIB; else export LGM_AMD_LIB=$V/lib_$n.so; fi
    timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cfg4 --no-cfg5 --no-attention --no-cpu-baseline --no-det > gpurun_out/r5g/b_${n}_r${round}.json 2> gpurun_out/r5g/b_${n}_r${round}.err || exit $?
    python -c "
import json
b=json.load(open('gpurun_out/r5g/b_${n}_r${round}.json')); c=b['cfg3_view_sharded']
print('$n r$round pool', b['ms_per_step'], {k: v['avg_us'] for k, v in b['kernels'].items() if k=='k_render_bwd'}, 'cfg3', c['ms_per_step'], {k: v['avg_us'] for k, v in c['kernels'].items() if k=='k_render_bwd'})"
  done
done
