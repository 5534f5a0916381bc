#!/bin/bash
# Round-5 session AL: MVAttention's GroupNorm kernels with their per-thread load loops batched 8 deep (k_mva_gn_tok's
# slab loads, k_mva_gn_coef's tile partials; LGM_MVA_BATCH=1: lib_mb1) against HEAD (lib_mb0), sums in the same
# order: attention GPU tests on mb1, then scripts/bench_mva.py and scripts/diag_cfg4.py per library, two rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5al
V=$PWD/lgm_amd/_lib/variants_attn
LGM_AMD_LIB=$V/lib_mb1.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/r5al/t_attn_mb1.log 2>&1
rc=$?; echo "mb1 tests: $(tail -1 gpurun_out/r5al/t_attn_mb1.log)"; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for n in mb0 mb1; do
    LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 300 python scripts/bench_mva.py > gpurun_out/r5al/mva_${n}_r${round}.json 2> gpurun_out/r5al/mva_${n}_r${round}.err || exit $?
    echo "$n r$round $(cat gpurun_out/r5al/mva_${n}_r${round}.json)"
    LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 300 python scripts/diag_cfg4.py > gpurun_out/r5al/cfg4_${n}_r${round}.json 2> gpurun_out/r5al/cfg4_${n}_r${round}.err || exit $?
    echo "$n r$round cfg4 $(head -c 400 gpurun_out/r5al/cfg4_${n}_r${round}.json)"
  done
done
