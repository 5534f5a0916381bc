#!/bin/bash
# Round-4 session F: (1) attention tests + kernel times at HEAD (coalesced delta rows, dK/dV row statistics stored
# negated); (2) three render A/B arms against lib_base: lib_hb (backward half-batch tail), lib_spair (two small
# tiles per sort workgroup), lib_priv (per-workgroup count rows: no memset, no reservation atomics): output hashes,
# the render tests on each arm, three interleaved A/B rounds of pool + cfg3 kernel times.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V=$PWD/lgm_amd/_lib/variants
step() { echo "== $1 $(date +%s)"; }
ab() {  # $1 variant, $2 round
  LGM_AMD_LIB=$V/lib_$1.so timeout -k 10 150 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-attention --no-cfg4 --no-cfg5 --no-det > gpurun_out/ab_$1_r$2.json 2>/dev/null || return $?
  python -c "import json;b=json.load(open('gpurun_out/ab_$1_r$2.json'));c=b['cfg3_view_sharded'];print('$1 r$2', b['ms_per_step'], {k:v['avg_us'] for k,v in b['kernels'].items()}, 'cfg3', c['ms_per_step'], c['step_spread']['median_ms'], {k:v['avg_us'] for k,v in c['kernels'].items()})"
}
step attn_tests
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/t_attn.log 2>&1
ra=$?; tail -2 gpurun_out/t_attn.log; [ $ra -eq 0 ] || [ $ra -eq 1 ] || exit $ra
step attn_bench
timeout -k 10 200 python scripts/bench_attn.py --no-sdpa --iters 20 > gpurun_out/attn_r4f.jsonl 2>/dev/null || exit $?
python -c "
import json
for l in open('gpurun_out/attn_r4f.jsonl'):
    r=json.loads(l); print(r['level'], 'fwd %.0f TF fwdbwd %.0f TF' % (r['fwd_tflops'], r['fwdbwd_tflops']), {k: round(v, 3) for k, v in r['kernels_ms'].items()})"
for v in base hb spair priv bin448 priv448; do step hash_$v; LGM_AMD_LIB=$V/lib_$v.so timeout -k 10 120 python scripts/render_hashes.py 2>/dev/null | tail -1 > gpurun_out/hash_$v.json || exit $?; cat gpurun_out/hash_$v.json; done
rc=0
for v in hb spair priv priv448; do
  step tests_$v
  LGM_AMD_LIB=$V/lib_$v.so timeout -k 10 420 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_render_parity_gpu.py tests/test_render_gpu.py tests/test_loss_gpu.py > gpurun_out/t_$v.log 2>&1
  r=$?; tail -2 gpurun_out/t_$v.log; [ $r -eq 0 ] || [ $r -eq 1 ] || exit $r; rc=$((rc | r))
done
for r in 1 2 3; do for v in base hb spair priv bin448 priv448; do step "ab $v r$r"; ab $v $r || exit $?; done; done
# (3) attention: the tile bodies split into two 32-key / 32-query halves (asplit), and dK,dV held at 4 waves per
# SIMD (asplit4), against abase (HEAD)
for r in 1 2; do for v in abase asplit asplit4; do
  step "attn $v r$r"; LGM_AMD_LIB=$V/lib_$v.so timeout -k 10 200 python scripts/bench_attn.py --no-sdpa --iters 20 > gpurun_out/attn_${v}_r$r.jsonl 2>/dev/null || exit $?
  python -c "
import json
for l in open('gpurun_out/attn_${v}_r$r.jsonl'):
    r=json.loads(l); print('$v', r['level'], 'fwd %.0f fwdbwd %.0f' % (r['fwd_tflops'], r['fwdbwd_tflops']), {k: round(v, 3) for k, v in r['kernels_ms'].items()})"
done; done
for v in asplit asplit4; do
  step tests_$v
  LGM_AMD_LIB=$V/lib_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/t_$v.log 2>&1
  r=$?; tail -2 gpurun_out/t_$v.log; [ $r -eq 0 ] || [ $r -eq 1 ] || exit $r; rc=$((rc | r))
done
exit $((ra | rc))
