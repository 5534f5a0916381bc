#!/bin/bash
# Round-5 session Q: the forward's and dQ's key-tile loops run as the two LDS buffers' bodies in turn as well
# (lib_unr; lib_kvu: dK,dV only; lib_base: HEAD): attention GPU tests on unr, then scripts/attn_ab.py, two rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5q
V=$PWD/lgm_amd/_lib/variants_attn
LGM_AMD_LIB=$V/lib_unr.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/r5q/t_attn_unr.log 2>&1
rc=$?; echo "unr tests: $(tail -1 gpurun_out/r5q/t_attn_unr.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u scripts/attn_ab.py > gpurun_out/r5q/ab.txt 2>&1
rc=$?; cat gpurun_out/r5q/ab.txt; exit $rc
