#!/bin/bash
# Round-4 session Z: the attention forward's row-sum MFMAs moved after the last sub-tile's rescale check (lib_reord),
# plus an MFMA / VALU interleave request (lib_iglp: sched_group_barrier), vs lib_base: attention GPU tests on both
# variants, then scripts/bench_attn.py, three rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
V=$PWD/lgm_amd/_lib/variants
for n in reord iglp; do
  echo "== tests $n $(date +%s)"
  LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/t_attn_$n.log 2>&1
  rc=$?; tail -1 gpurun_out/t_attn_$n.log; [ $rc -eq 0 ] || exit $rc
done
for round in 1 2 3; do
  for n in base reord iglp; do
    LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 200 python scripts/bench_attn.py --no-sdpa --iters 20 > gpurun_out/ab/attn_${n}_r${round}.jsonl 2>/dev/null || exit $?
    python -c "
import json
for l in open('gpurun_out/ab/attn_${n}_r${round}.jsonl'):
    r=json.loads(l); print('$n r$round', r['level'], 'fwd %.0f TF fwdbwd %.0f TF' % (r['fwd_tflops'], r['fwdbwd_tflops']), {k: round(v, 3) for k, v in r['kernels_ms'].items()})" | grep -E "c512_32x32|c512_40x40"
  done
done
