#!/bin/bash
# Round-5 session AP: k_mva_gn_reg with one item per thread where that covers the slab (58 VGPRs; LGM_GNR_K1=1:
# lib_k1) against two (lib_k0): attention GPU tests on k1, then scripts/bench_mva.py and
# scripts/diag_cfg4.py per library, two rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5ap
V=$PWD/lgm_amd/_lib/variants_attn
LGM_AMD_LIB=$V/lib_k1.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/r5ap/t_attn_k1.log 2>&1
rc=$?; echo "k1 tests: $(tail -1 gpurun_out/r5ap/t_attn_k1.log)"; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for n in k0 k1; do
    LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 300 python scripts/bench_mva.py > gpurun_out/r5ap/mva_${n}_r${round}.json 2> gpurun_out/r5ap/mva_${n}_r${round}.err || exit $?
    echo "$n r$round $(cat gpurun_out/r5ap/mva_${n}_r${round}.json)"
    LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 300 python scripts/diag_cfg4.py > gpurun_out/r5ap/cfg4_${n}_r${round}.json 2> gpurun_out/r5ap/cfg4_${n}_r${round}.err || exit $?
    echo "$n r$round cfg4 $(head -c 400 gpurun_out/r5ap/cfg4_${n}_r${round}.json)"
  done
done
