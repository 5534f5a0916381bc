#!/bin/bash
# Round-5 session W: MVAttention's GroupNorm -> tokens in one launch per (group, sample) with the slab in LDS
# (lib_gnf, LGM_MVA_GN_FUSED) against the chunked statistics + tiled normalise launches (lib_base, HEAD):
# the attention tests on gnf (fused-vs-torch MVAttention, module fixtures), then scripts/diag_cfg4.py per library,
# two interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5w
V=$PWD/lgm_amd/_lib/variants
LGM_AMD_LIB=$V/lib_gnf.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/r5w/t_attn_gnf.log 2>&1
rc=$?; echo "gnf tests: $(tail -1 gpurun_out/r5w/t_attn_gnf.log)"; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for n in base gnf; do
    LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 300 python scripts/diag_cfg4.py > gpurun_out/r5w/cfg4_${n}_r${round}.txt 2> gpurun_out/r5w/cfg4_${n}_r${round}.err || exit $?
    echo "$n r$round $(head -1 gpurun_out/r5w/cfg4_${n}_r${round}.txt)"
  done
done
