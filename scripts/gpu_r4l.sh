#!/bin/bash
# Round-4 session M: the D = 32 attention forward with four query sub-tiles per wave at 2 waves per SIMD (lib_afuse)
# vs lib_abase: bench_attn kernel times (three rounds), then the attention tests on lib_afuse.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V=$PWD/lgm_amd/_lib/variants
step() { echo "== $1 $(date +%s)"; }
for r in 1 2 3; do for v in abase afuse; do
  step "attn $v r$r"; LGM_AMD_LIB=$V/lib_$v.so timeout -k 10 200 python scripts/bench_attn.py --no-sdpa --iters 20 > gpurun_out/attn_${v}_r$r.jsonl 2>/dev/null || exit $?
  python -c "
import json
for l in open('gpurun_out/attn_${v}_r$r.jsonl'):
    r=json.loads(l); print('$v', r['level'], 'fwd %.0f fwdbwd %.0f' % (r['fwd_tflops'], r['fwdbwd_tflops']), {k: round(v, 3) for k, v in r['kernels_ms'].items()})"
done; done
step tests_afuse
LGM_AMD_LIB=$V/lib_afuse.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/t_afuse.log 2>&1
rc=$?; tail -2 gpurun_out/t_afuse.log
exit $rc
