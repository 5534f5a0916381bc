#!/bin/bash
# Round-5 session B: dK/dV recomputing P from the forward's rounded operand (Q * c in a second LDS image, lib = HEAD)
# vs K * c (lib_kpre): the per-output error record vs fp64, the attention GPU tests, then scripts/bench_attn.py.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5b
V=$PWD/lgm_amd/_lib/variants
LGM_AMD_LIB=$V/lib_kpre.so timeout -k 10 300 python scripts/diag_attn_precision.py > gpurun_out/r5b/prec_kpre.jsonl 2> gpurun_out/r5b/prec_kpre.err || exit $?
timeout -k 10 300 python scripts/diag_attn_precision.py > gpurun_out/r5b/prec_head.jsonl 2> gpurun_out/r5b/prec_head.err || exit $?
cat gpurun_out/r5b/prec_*.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/r5b/t_attn.log 2>&1
rc=$?; tail -1 gpurun_out/r5b/t_attn.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for n in kpre head; do
    if [ $n = head ]; then unset LGM_AMD_LIB; else export LGM_AMD_LIB=$V/lib_$n.so; fi
    timeout -k 10 200 python scripts/bench_attn.py --no-sdpa --iters 20 > gpurun_out/r5b/attn_${n}_r${round}.jsonl 2>/dev/null || exit $?
    python -c "
import json
for l in open('gpurun_out/r5b/attn_${n}_r${round}.jsonl'):
    r=json.loads(l); print('$n r$round', r['level'], 'fwd %.0f TF fwdbwd %.0f TF' % (r['fwd_tflops'], r['fwdbwd_tflops']), {k: round(v, 3) for k, v in r['kernels_ms'].items()})"
  done
done
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_render_gpu.py tests/test_head.py -m gpu -k "needle or saturation or retain or head" > gpurun_out/r5b/t_render_new.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r5b/t_render_new.log | tail -30; grep "^head " gpurun_out/r5b/t_render_new.log | head -60; [ $rc -eq 0 ] || exit $rc
# backward section shares (LGM_BWD_STAMPS build) on the pool and one scene, and the single scene's work timelines
LGM_AMD_LIB=$PWD/lgm_amd/_lib/variants/lib_stamps.so timeout -k 10 200 python scripts/diag_bwd_stamps.py 8 > gpurun_out/r5b/stamps_B8.json 2>&1 || exit $?
LGM_AMD_LIB=$PWD/lgm_amd/_lib/variants/lib_stamps.so timeout -k 10 200 python scripts/diag_bwd_stamps.py 1 > gpurun_out/r5b/stamps_B1.json 2>&1 || exit $?
tail -1 gpurun_out/r5b/stamps_B8.json; tail -1 gpurun_out/r5b/stamps_B1.json
timeout -k 10 200 python scripts/diag_counters.py 1 > gpurun_out/r5b/counters_B1.log 2>&1 || exit $?
tail -5 gpurun_out/r5b/counters_B1.log | cut -c1-600
