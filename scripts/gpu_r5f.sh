#!/bin/bash
# Round-5 session F: k_render_bwd section shares at 8 sections (LGM_BWD_STAMPS build: the barriers and the DMA wait
# apart) on the pool and on one scene; the new attention error-record and MVAttention fused-backward tests.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5f
LGM_AMD_LIB=$PWD/lgm_amd/_lib/variants/lib_stamps.so timeout -k 10 200 python scripts/diag_bwd_stamps.py 8 > gpurun_out/r5f/stamps_B8.json 2>&1 || exit $?
LGM_AMD_LIB=$PWD/lgm_amd/_lib/variants/lib_stamps.so timeout -k 10 200 python scripts/diag_bwd_stamps.py 1 > gpurun_out/r5f/stamps_B1.json 2>&1 || exit $?
tail -1 gpurun_out/r5f/stamps_B8.json; tail -1 gpurun_out/r5f/stamps_B1.json
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_attention.py -m gpu -k "error_record or mvattention" > gpurun_out/r5f/t_attn.log 2>&1
rc=$?; grep -E "passed|failed|error record|mva fused" gpurun_out/r5f/t_attn.log | tail -20; exit $rc
