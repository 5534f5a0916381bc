#!/bin/bash
# Round-5 session D: k_render_bwd with per-wave conversion + flush (lib_wflush: one barrier per chunk) vs HEAD:
# the render GPU tests on the variant, then bench.py's pool and single scene, two interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5d
V=$PWD/lgm_amd/_lib/variants
LGM_AMD_LIB=$V/lib_wflush.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_render_gpu.py tests/test_render_parity_gpu.py tests/test_training_gpu.py -m gpu > gpurun_out/r5d/t_render_wflush.log 2>&1
rc=$?; tail -2 gpurun_out/r5d/t_render_wflush.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for n in head wflush; do
    if [ $n = head ]; then unset LGM_AMD_LIB; else export LGM_AMD_LIB=$V/lib_$n.so; fi
    timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cfg4 --no-cfg5 --no-attention --no-cpu-baseline --no-det > gpurun_out/r5d/b_${n}_r${round}.json 2> gpurun_out/r5d/b_${n}_r${round}.err || exit $?
    python -c "
import json
b=json.load(open('gpurun_out/r5d/b_${n}_r${round}.json')); c=b['cfg3_view_sharded']
print('$n r$round pool', b['ms_per_step'], b['step_spread']['median_ms'], {k: v['avg_us'] for k, v in b['kernels'].items()}, 'cfg3', c['ms_per_step'], c['step_spread']['median_ms'], {k: v['avg_us'] for k, v in c['kernels'].items()})"
  done
done
python -c "import json; print(json.dumps(json.load(open('gpurun_out/grad_precision.json')))[:3000])" 2>/dev/null
