#!/bin/bash
# Round-5 session N: (1) D = 32: 4 query sub-tiles per forward wave at 3 (fq4, 2 VGPRs spilled) or 2 (fq4w2) waves
# per SIMD, dK,dV with 3 key sub-tiles at 3 waves (kv3w3), both (fq4kv3), against the working tree (base):
# attention GPU tests on kv3w3 and fq4kv3, then scripts/attn_ab.py. (2) D = 64 LDS-DMA staging (d64dma, this tree)
# against HEAD's register staging (d64reg): attention GPU tests on d64dma, then scripts/bench_attn.py per library,
# two interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5n
V=$PWD/lgm_amd/_lib/variants_attn
V64=$PWD/lgm_amd/_lib/variants_attn64
for lib in $V/lib_kv3w3.so $V/lib_fq4kv3.so $V64/lib_d64dma.so; do
  n=$(basename $lib .so)
  LGM_AMD_LIB=$lib timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/r5n/t_$n.log 2>&1
  rc=$?; echo "$n tests: $(tail -1 gpurun_out/r5n/t_$n.log)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 python -u scripts/attn_ab.py > gpurun_out/r5n/ab.txt 2>&1
rc=$?; cat gpurun_out/r5n/ab.txt; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for n in d64reg d64dma; do
    LGM_AMD_LIB=$V64/lib_$n.so timeout -k 10 300 python scripts/bench_attn.py --no-sdpa --iters 20 > gpurun_out/r5n/attn_${n}_r${round}.jsonl 2> gpurun_out/r5n/attn_${n}_r${round}.err || exit $?
    python -c "
import json
for l in open('gpurun_out/r5n/attn_${n}_r${round}.jsonl'):
    r=json.loads(l); print('$n r$round', r['level'], 'fwd %.0f TF fwdbwd %.0f TF' % (r['fwd_tflops'], r['fwdbwd_tflops']), {k: round(1e3*v, 1) for k, v in r['kernels_ms'].items()})"
  done
done
