#!/bin/bash
# Round-5 session I: the small-tile sort (lib_sortsmall: k_sort_small for lists <= 2,016 at 8 workgroups per CU,
# k_sort for the rest) -- render GPU tests on it (bit-exact tile lists, ties, clustered depths), bench.py pool +
# single scene vs HEAD, two interleaved rounds; then the first-step host latency probe.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5i
V=$PWD/lgm_amd/_lib/variants
LGM_AMD_LIB=$V/lib_sortsmall.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_render_gpu.py tests/test_render_parity_gpu.py -m gpu > gpurun_out/r5i/t_render_ss.log 2>&1
rc=$?; tail -1 gpurun_out/r5i/t_render_ss.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for n in head sortsmall; do
    if [ $n = head ]; then unset LGM_AMD_LIB; else export LGM_AMD_LIB=$V/lib_$n.so; fi
    timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cfg4 --no-cfg5 --no-attention --no-cpu-baseline --no-det > gpurun_out/r5i/b_${n}_r${round}.json 2> gpurun_out/r5i/b_${n}_r${round}.err || exit $?
    python -c "
import json
b=json.load(open('gpurun_out/r5i/b_${n}_r${round}.json')); c=b['cfg3_view_sharded']
print('$n r$round pool', b['ms_per_step'], {k: v['avg_us'] for k, v in b['kernels'].items()}, 'cfg3', c['ms_per_step'], {k: v['avg_us'] for k, v in c['kernels'].items()})"
  done
done
unset LGM_AMD_LIB
timeout -k 10 200 python scripts/diag_first_step.py --iters 20 > gpurun_out/r5i/first_step.json 2>&1 || exit $?
cat gpurun_out/r5i/first_step.json
