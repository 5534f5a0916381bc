#!/bin/bash
# Round-5 session Z: s_setprio(1) around every attention MFMA cluster (LGM_ATTN_PRIO: lib_prio) against HEAD
# (lib_base): attention GPU tests on prio, then scripts/attn_ab.py, two rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5z
V=$PWD/lgm_amd/_lib/variants_attn
LGM_AMD_LIB=$V/lib_prio.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/r5z/t_attn_prio.log 2>&1
rc=$?; echo "prio tests: $(tail -1 gpurun_out/r5z/t_attn_prio.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u scripts/attn_ab.py > gpurun_out/r5z/ab.txt 2>&1
rc=$?; cat gpurun_out/r5z/ab.txt; exit $rc
