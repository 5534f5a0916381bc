#!/bin/bash
# Round-4 session W: dK,dV with its per-tile LDS row address recomputed instead of spilled (lib_dkfix) vs lib_base:
# attention GPU tests on lib_dkfix, then scripts/bench_attn.py (HIP kernels) on both, three rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
V=$PWD/lgm_amd/_lib/variants
echo "== tests $(date +%s)"
LGM_AMD_LIB=$V/lib_dkfix.so timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/t_attn.log 2>&1
rc=$?; tail -2 gpurun_out/t_attn.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do
  for n in base dkfix; do
    LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 200 python scripts/bench_attn.py --no-sdpa --iters 20 > gpurun_out/ab/attn_${n}_r${round}.jsonl 2>/dev/null || exit $?
    python -c "
import json
for l in open('gpurun_out/ab/attn_${n}_r${round}.jsonl'):
    r=json.loads(l); print('$n r$round', r['level'], 'fwd %.0f TF fwdbwd %.0f TF' % (r['fwd_tflops'], r['fwdbwd_tflops']), {k: round(v, 3) for k, v in r['kernels_ms'].items()})" | head -2
  done
done
