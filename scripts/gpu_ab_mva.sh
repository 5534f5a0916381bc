#!/bin/bash
# Attention-side A/B: bench.py --only-attn (attention level, MVAttention level, cfg4) per variant library in $AB_LIBS
# (default: every lgm_amd/_lib/variants/lib_*.so), 2 interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
AB=${OUTAB:-gpurun_out/ab}; mkdir -p $AB
LIBS=${AB_LIBS:-$(ls lgm_amd/_lib/variants/lib_*.so)}
for round in 1 2; do
  for lib in $LIBS; do
    n=$(basename $lib .so)
    LGM_AMD_LIB=$PWD/$lib timeout -k 10 200 python bench.py --only-attn --steps 10 > $AB/mva_${n}_r${round}.json 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; exit $rc; }
    python -c "
import json
b = json.load(open('$AB/mva_${n}_r${round}.json')); m = b['mva_level']
print('$n r$round', 'mva', m['fused_ms'], {k: v['avg_us'] for k, v in m['kernels'].items()}, 'attn', b['attention']['tflops'], 'cfg4', b['cfg4']['attention_ms'])"
  done
done
