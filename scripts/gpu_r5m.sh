#!/bin/bash
# Round-5 session M: D = 32 attention with 3 / 4 query sub-tiles per forward wave (fq3, fq4) and 3 per dQ wave
# (dq3) against HEAD (base, 2 each): attention GPU tests on fq4 and dq3, then scripts/attn_ab.py, two rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5m
V=$PWD/lgm_amd/_lib/variants_attn
for n in fq4 dq3; do
  LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/r5m/t_attn_$n.log 2>&1
  rc=$?; echo "$n tests: $(tail -1 gpurun_out/r5m/t_attn_$n.log)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 python -u scripts/attn_ab.py > gpurun_out/r5m/ab.txt 2>&1
rc=$?; cat gpurun_out/r5m/ab.txt; exit $rc
