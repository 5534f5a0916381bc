#!/bin/bash
# Round-5 session L: the D = 32 attention forward with LDS-DMA K/V staging on a swizzled unpadded image
# (LGM_ATTN_FWD_DMA) and/or held at 5 waves per SIMD (LGM_ATTN_FWD_WPE32=5): attention GPU tests on the DMA
# variants, then scripts/attn_ab.py (bench level per-kernel times + output/gradient hashes), two rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5l
V=$PWD/lgm_amd/_lib/variants_attn
for n in dma5 alldma; do
  LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/r5l/t_attn_$n.log 2>&1
  rc=$?; echo "$n tests: $(tail -1 gpurun_out/r5l/t_attn_$n.log)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 python -u scripts/attn_ab.py > gpurun_out/r5l/ab.txt 2>&1
rc=$?; cat gpurun_out/r5l/ab.txt; exit $rc
