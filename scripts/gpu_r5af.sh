#!/bin/bash
# Round-5 session AF: the D = 32 forward on v_mfma_f32_32x32x16 (k_attn_fwd3, LGM_ATTN_FWD3=1: lib_f31) against the
# 16x16x32 k_attn_fwd2 (lib_f30): attention GPU tests on f31, then scripts/attn_ab.py (bench level, two rounds) and
# scripts/diag_cfg4.py per library.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5af
V=$PWD/lgm_amd/_lib/variants_attn
LGM_AMD_LIB=$V/lib_f31.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/r5af/t_attn_f31.log 2>&1
rc=$?; echo "f31 tests: $(tail -1 gpurun_out/r5af/t_attn_f31.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u scripts/attn_ab.py > gpurun_out/r5af/ab.txt 2>&1
rc=$?; cat gpurun_out/r5af/ab.txt; [ $rc -eq 0 ] || exit $rc
for n in f30 f31; do
  LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 300 python scripts/diag_cfg4.py > gpurun_out/r5af/cfg4_$n.json 2> gpurun_out/r5af/cfg4_$n.err || exit $?
  echo "$n cfg4 $(head -c 600 gpurun_out/r5af/cfg4_$n.json)"
done
