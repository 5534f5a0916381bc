#!/bin/bash
# Interleaved A/B timing of variant libraries (built here, shipped in the snapshot): 2 rounds per variant.
cd "$GRAFT_REPO_ROOT" || exit 1
AB=${OUTAB:-gpurun_out/ab}; mkdir -p $AB
for round in 1 2; do
  for lib in ${AB_LIBS:-lgm_amd/_lib/variants/lib_*.so}; do
    n=$(basename $lib .so)
    LGM_AMD_LIB=$PWD/$lib timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-attention --no-cfg4 --no-cfg5 > $AB/${n}_r${round}.json 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; exit $rc; }
    if [ $round -eq 1 ]; then  # output hashes (variants meant to be bitwise equal must print the same)
      LGM_AMD_LIB=$PWD/$lib timeout -k 10 120 python scripts/render_hashes.py > $AB/${n}_hash.json 2>/dev/null
      rc=$?; [ $rc -eq 0 ] || { echo "$n hashes failed rc=$rc"; exit $rc; }
      echo "$n hashes $(cat $AB/${n}_hash.json)"
    fi
    python -c "import json;b=json.load(open('$AB/${n}_r${round}.json'));c3=b['cfg3_view_sharded'];dt=b.get('deterministic') or {};print('$n', 'r$round', b['ms_per_step'], {k:v['avg_us'] for k,v in b['kernels'].items()}, 'cfg3', c3['ms_per_step'], {k:v['avg_us'] for k,v in c3.get('kernels',{}).items()}, 'cfg2', (b.get('cfg2') or {}).get('ms_per_step'), (b.get('cfg2') or {}).get('gpu_span_ms_per_step'), {k:v['avg_us'] for k,v in (b.get('cfg2') or {}).get('kernels',{}).items()}, 'det', dt.get('ms_per_step'), {k:v['avg_us'] for k,v in dt.get('kernels',{}).items()})"
  done
done
