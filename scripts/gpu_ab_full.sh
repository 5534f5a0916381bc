#!/bin/bash
# Interleaved A/B of variant libraries on the full default bench line minus the attention / CPU legs (pool, cfg3,
# cfg2, cfg4's render, cfg5's render side, deterministic pool): 2 rounds per variant.
cd "$GRAFT_REPO_ROOT" || exit 1
AB=${OUTAB:-gpurun_out/abfull}; mkdir -p $AB
for round in 1 2; do
  for lib in ${AB_LIBS:-lgm_amd/_lib/variants/lib_*.so}; do
    n=$(basename $lib .so)
    LGM_AMD_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-attention > $AB/${n}_r${round}.json 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; exit $rc; }
    python -c "import json;b=json.load(open('$AB/${n}_r${round}.json'));c3=b['cfg3_view_sharded'];c4=b.get('cfg4') or {};c5=b.get('cfg5') or {};print('$n', 'r$round', b['ms_per_step'], {k:v['avg_us'] for k,v in b['kernels'].items()}, 'cfg3', c3['ms_per_step'], {k:v['avg_us'] for k,v in c3.get('kernels',{}).items()}, 'cfg4', {k:v for k,v in c4.items() if 'render' in k and not isinstance(v,dict)}, 'cfg5', {k:v for k,v in c5.items() if not isinstance(v,(dict,list))})"
  done
done
