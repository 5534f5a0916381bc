#!/bin/bash
# Round-4 session P: the compiler's machine-scheduler strategy (-mllvm -amdgpu-sched-strategy = max-ilp or
# max-memory-clause; iterative-ilp crashes the compiler on attention.hip) for the whole library vs the default (lib_base): hashes (expected bitwise
# equal), three render A/B rounds, one attention round.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
V=$PWD/lgm_amd/_lib/variants
VARS="base ilp mclause"
step() { echo "== $1 $(date +%s)"; }
ab() {  # $1 variant, $2 round
  LGM_AMD_LIB=$V/lib_$1.so timeout -k 10 150 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-attention --no-cfg4 --no-cfg5 --no-det > gpurun_out/ab_$1_r$2.json 2>/dev/null || return $?
  python -c "import json;b=json.load(open('gpurun_out/ab_$1_r$2.json'));c=b['cfg3_view_sharded'];print('$1 r$2', b['ms_per_step'], {k:v['avg_us'] for k,v in b['kernels'].items()}, 'cfg3', c['ms_per_step'], c['step_spread']['median_ms'], {k:v['avg_us'] for k,v in c['kernels'].items()})"
}
for v in $VARS; do step hash_$v; LGM_AMD_LIB=$V/lib_$v.so timeout -k 10 120 python scripts/render_hashes.py 2>/dev/null | tail -1 > gpurun_out/hash_$v.json || exit $?; cat gpurun_out/hash_$v.json; done
for r in 1 2 3; do for v in $VARS; do step "ab $v r$r"; ab $v $r || exit $?; done; done
for v in $VARS; do
  step "attn $v"
  LGM_AMD_LIB=$V/lib_$v.so timeout -k 10 200 python scripts/bench_attn.py --no-sdpa --iters 20 > gpurun_out/ab/attn_$v.jsonl 2>/dev/null || exit $?
  python -c "
import json
for l in open('gpurun_out/ab/attn_$v.jsonl'):
    r=json.loads(l); print('$v', r['level'], 'fwd %.0f TF fwdbwd %.0f TF' % (r['fwd_tflops'], r['fwdbwd_tflops']), {k: round(v, 3) for k, v in r['kernels_ms'].items()})"
done
