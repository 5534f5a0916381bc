#!/bin/bash
# Round-5 session P: dK,dV's query-tile loop run as the two LDS buffers' bodies in turn (compile-time buffer index,
# per-lane DMA source offsets kept across tiles: lib_kvu) against HEAD (lib_base): attention GPU tests on kvu, then
# scripts/attn_ab.py (bench level per-kernel times + hashes), two rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5p
V=$PWD/lgm_amd/_lib/variants_attn
LGM_AMD_LIB=$V/lib_kvu.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/r5p/t_attn_kvu.log 2>&1
rc=$?; echo "kvu tests: $(tail -1 gpurun_out/r5p/t_attn_kvu.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u scripts/attn_ab.py > gpurun_out/r5p/ab.txt 2>&1
rc=$?; cat gpurun_out/r5p/ab.txt; exit $rc
