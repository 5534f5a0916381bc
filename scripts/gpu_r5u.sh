#!/bin/bash
# Round-5 session U: the two-sub-tile D = 32 forward (cfg4's L = 9600: 1,200 workgroups) held at 5 waves per SIMD
# (1,280 slots: one round instead of 1.17; lib_q2w5) against HEAD (lib_base): attention GPU tests on q2w5, then
# scripts/bench_attn.py per library, two interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5u
V64=$PWD/lgm_amd/_lib/variants_attn64
LGM_AMD_LIB=$V64/lib_q2w5.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/r5u/t_attn.log 2>&1
rc=$?; echo "tests: $(tail -1 gpurun_out/r5u/t_attn.log)"; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for n in base q2w5; do
    LGM_AMD_LIB=$V64/lib_$n.so timeout -k 10 300 python scripts/bench_attn.py --no-sdpa --iters 20 > gpurun_out/r5u/attn_${n}_r${round}.jsonl 2> gpurun_out/r5u/attn_${n}_r${round}.err || exit $?
    python -c "
import json
for l in open('gpurun_out/r5u/attn_${n}_r${round}.jsonl'):
    r=json.loads(l); print('$n r$round', r['level'], 'fwd %.0f TF fwdbwd %.0f TF' % (r['fwd_tflops'], r['fwdbwd_tflops']), {k: round(1e3*v, 1) for k, v in r['kernels_ms'].items()})"
  done
done
