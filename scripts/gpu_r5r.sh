#!/bin/bash
# Round-5 session R: dK,dV's per-row constants (-lse', -delta) written by k_attn_dq2 and DMA'd with each query tile
# (lib_rowdma) against HEAD (lib_base): attention GPU tests on rowdma, then scripts/attn_ab.py, two rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5r
V=$PWD/lgm_amd/_lib/variants_attn
LGM_AMD_LIB=$V/lib_rowdma.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/r5r/t_attn_rowdma.log 2>&1
rc=$?; echo "rowdma tests: $(tail -1 gpurun_out/r5r/t_attn_rowdma.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u scripts/attn_ab.py > gpurun_out/r5r/ab.txt 2>&1
rc=$?; cat gpurun_out/r5r/ab.txt; exit $rc
