#!/bin/bash
# Round-5 session S: the forward without a per-tile row max (the row sum checked after the tile's exponentials,
# LGM_ATTN_LATE_CHECK, with per-issue DMA lane offsets LGM_ATTN_FRESH_DMA: lib_late), the lane offsets alone
# (lib_fresh), HEAD (lib_base): the new score-jump test on base, all attention GPU tests on late, then
# scripts/attn_ab.py, two rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5s
V=$PWD/lgm_amd/_lib/variants_attn
LGM_AMD_LIB=$V/lib_base.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py -m gpu -k score_jump > gpurun_out/r5s/t_jump_base.log 2>&1
rc=$?; echo "base jump tests: $(tail -1 gpurun_out/r5s/t_jump_base.log)"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
LGM_AMD_LIB=$V/lib_late.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/r5s/t_attn_late.log 2>&1
rc=$?; echo "late tests: $(tail -1 gpurun_out/r5s/t_attn_late.log)"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u scripts/attn_ab.py > gpurun_out/r5s/ab.txt 2>&1
rc=$?; cat gpurun_out/r5s/ab.txt; exit $rc
