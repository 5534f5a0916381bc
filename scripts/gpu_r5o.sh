#!/bin/bash
# Round-5 session O: the D = 32 forward with 4 query sub-tiles per wave wherever its grid has >= 512 workgroups
# (lib_qs4 = this tree) against 2 (lib_d64dma): attention GPU tests on this tree's library, then
# scripts/bench_attn.py per library (every LGM level incl. cfg4's L = 9600), two interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5o
V64=$PWD/lgm_amd/_lib/variants_attn64
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/r5o/t_attn.log 2>&1
rc=$?; echo "tests: $(tail -1 gpurun_out/r5o/t_attn.log)"; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for n in d64dma qs4; do
    LGM_AMD_LIB=$V64/lib_$n.so timeout -k 10 300 python scripts/bench_attn.py --no-sdpa --iters 20 > gpurun_out/r5o/attn_${n}_r${round}.jsonl 2> gpurun_out/r5o/attn_${n}_r${round}.err || exit $?
    python -c "
import json
for l in open('gpurun_out/r5o/attn_${n}_r${round}.jsonl'):
    r=json.loads(l); print('$n r$round', r['level'], 'fwd %.0f TF fwdbwd %.0f TF' % (r['fwd_tflops'], r['fwdbwd_tflops']), {k: round(1e3*v, 1) for k, v in r['kernels_ms'].items()})"
  done
done
