#!/bin/bash
# Round-5 session C2: dK/dV reading the Q * c rows k_attn_dq2 wrote (HEAD): error record vs fp64, attention GPU tests,
# scripts/bench_attn.py x2; then session D (scripts/gpu_r5d.sh: the wave-flush backward A/B).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5c
timeout -k 10 300 python scripts/diag_attn_precision.py > gpurun_out/r5c/prec_dqqc.jsonl 2> gpurun_out/r5c/prec_dqqc.err || exit $?
cat gpurun_out/r5c/prec_dqqc.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_attention.py tests/test_abi.py -m gpu > gpurun_out/r5c/t_attn.log 2>&1
rc=$?; tail -1 gpurun_out/r5c/t_attn.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  timeout -k 10 200 python scripts/bench_attn.py --no-sdpa --iters 20 > gpurun_out/r5c/attn_dqqc_r${round}.jsonl 2>/dev/null || exit $?
  python -c "
import json
for l in open('gpurun_out/r5c/attn_dqqc_r${round}.jsonl'):
    r=json.loads(l); print('dqqc r$round', r['level'], 'fwd %.0f TF fwdbwd %.0f TF' % (r['fwd_tflops'], r['fwdbwd_tflops']), {k: round(v, 3) for k, v in r['kernels_ms'].items()})" | grep -E "c512_32x32|c512_40x40"
done
bash scripts/gpu_r5d.sh || exit $?
