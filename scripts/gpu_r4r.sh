#!/bin/bash
# Round-4 session R: half-step checkpoints for small launches (lib_half: <= 2,048 tiles checkpoint every 128 list
# entries, twice the backward items) vs lib_base: hashes, render tests on lib_half, four A/B rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V=$PWD/lgm_amd/_lib/variants
VARS="base half"
step() { echo "== $1 $(date +%s)"; }
ab() {  # $1 variant, $2 round
  LGM_AMD_LIB=$V/lib_$1.so timeout -k 10 150 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-attention --no-cfg4 --no-cfg5 --no-det > gpurun_out/ab_$1_r$2.json 2>/dev/null || return $?
  python -c "import json;b=json.load(open('gpurun_out/ab_$1_r$2.json'));c=b['cfg3_view_sharded'];print('$1 r$2', b['ms_per_step'], {k:v['avg_us'] for k,v in b['kernels'].items()}, 'cfg3', c['ms_per_step'], c['step_spread']['median_ms'], {k:v['avg_us'] for k,v in c['kernels'].items()})"
}
for v in $VARS; do step hash_$v; LGM_AMD_LIB=$V/lib_$v.so timeout -k 10 120 python scripts/render_hashes.py 2>/dev/null | tail -1 > gpurun_out/hash_$v.json || exit $?; cat gpurun_out/hash_$v.json; done
step tests_half
LGM_AMD_LIB=$V/lib_half.so timeout -k 10 420 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_render_parity_gpu.py tests/test_render_gpu.py tests/test_loss_gpu.py tests/test_training_gpu.py > gpurun_out/t_half.log 2>&1
rc=$?; tail -3 gpurun_out/t_half.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2 3 4; do for v in $VARS; do step "ab $v r$r"; ab $v $r || exit $?; done; done
exit $rc
