#!/bin/bash
# Round-5 session H: k_render_bwd staging two chunks ahead (lib_dma2: chunk k + 2's DMA issued as soon as chunk k's
# records are released, wave 0 stages only, waves 1-3 flush, counted vmcnt) vs HEAD: render GPU tests on the variant,
# then bench.py pool + single scene, two interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5h
V=$PWD/lgm_amd/_lib/variants
LGM_AMD_LIB=$V/lib_dma2.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_render_gpu.py tests/test_render_parity_gpu.py tests/test_training_gpu.py tests/test_loss_gpu.py -m gpu > gpurun_out/r5h/t_render_dma2.log 2>&1
rc=$?; tail -1 gpurun_out/r5h/t_render_dma2.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for n in head dma2; do
    if [ $n = head ]; then unset LGM_AMD_LIB; else export LGM_AMD_LIB=$V/lib_$n.so; fi
    timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cfg4 --no-cfg5 --no-attention --no-cpu-baseline --no-det > gpurun_out/r5h/b_${n}_r${round}.json 2> gpurun_out/r5h/b_${n}_r${round}.err || exit $?
    python -c "
import json
b=json.load(open('gpurun_out/r5h/b_${n}_r${round}.json')); c=b['cfg3_view_sharded']
print('$n r$round pool', b['ms_per_step'], {k: v['avg_us'] for k, v in b['kernels'].items()}, 'cfg3', c['ms_per_step'], {k: v['avg_us'] for k, v in c['kernels'].items()})"
  done
done
