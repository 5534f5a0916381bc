#!/bin/bash
# Round-5 session AB: the backward with one 16-row sub-tile per wave (more waves per SIMD: dK,dV 5, dQ 6) for dK,dV
# (lib_kv1), dQ (lib_dq1), both (lib_both1) against HEAD (lib_base): tests on both1, then scripts/attn_ab.py.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5ab
V=$PWD/lgm_amd/_lib/variants_attn
LGM_AMD_LIB=$V/lib_both1.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/r5ab/t_attn_both1.log 2>&1
rc=$?; echo "both1 tests: $(tail -1 gpurun_out/r5ab/t_attn_both1.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u scripts/attn_ab.py > gpurun_out/r5ab/ab.txt 2>&1
rc=$?; cat gpurun_out/r5ab/ab.txt; exit $rc
