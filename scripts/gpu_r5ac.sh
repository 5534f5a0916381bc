#!/bin/bash
# Round-5 session AC: MVAttention's GroupNorm backward in one launch per (group, sample) with the x and dy slabs in
# LDS + a per-channel sum over samples (lib_gnb, LGM_MVA_GN_BWD_FUSED) against the part / coef / dx passes (lib_base):
# attention tests on gnb, then scripts/bench_mva.py per library, two interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5ac
V=$PWD/lgm_amd/_lib/variants
LGM_AMD_LIB=$V/lib_gnb.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/r5ac/t_attn_gnb.log 2>&1
rc=$?; echo "gnb tests: $(tail -1 gpurun_out/r5ac/t_attn_gnb.log)"; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for n in base gnb; do
    LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 300 python scripts/bench_mva.py > gpurun_out/r5ac/mva_${n}_r${round}.json 2> gpurun_out/r5ac/mva_${n}_r${round}.err || exit $?
    echo "$n r$round $(cat gpurun_out/r5ac/mva_${n}_r${round}.json)"
  done
done
