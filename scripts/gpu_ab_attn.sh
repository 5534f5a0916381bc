#!/bin/bash
# Attention A/B over the variant libraries: scripts/bench_attn.py (HIP kernels only) per library, 2 rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
AB=${OUTAB:-gpurun_out/ab}; mkdir -p $AB
for round in 1 2; do
  for lib in lgm_amd/_lib/variants/lib_*.so; do
    n=$(basename $lib .so)
    LGM_AMD_LIB=$PWD/$lib timeout -k 10 200 python scripts/bench_attn.py --no-sdpa --iters 20 > $AB/attn_${n}_r${round}.jsonl 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; exit $rc; }
    python -c "
import json
for l in open('$AB/attn_${n}_r${round}.jsonl'):
    r=json.loads(l); print('$n r$round', r['level'], 'fwd %.0f TF fwdbwd %.0f TF' % (r['fwd_tflops'], r['fwdbwd_tflops']), {k: round(v, 3) for k, v in r['kernels_ms'].items()})"
  done
done
