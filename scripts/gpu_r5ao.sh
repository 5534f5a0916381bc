#!/bin/bash
# Round-5 session AO: MVAttention's backward layout kernels with vector accesses (k_mva_out_bwd_v, k_mva_gn_part_v,
# k_mva_gn_dx_v; LGM_MVA_VECB=1: lib_vb1) against the scalar-width forms (lib_vb0): attention GPU tests on vb1, then
# scripts/bench_mva.py per library, two rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5ao
V=$PWD/lgm_amd/_lib/variants_attn
LGM_AMD_LIB=$V/lib_vb1.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/r5ao/t_attn_vb1.log 2>&1
rc=$?; echo "vb1 tests: $(tail -1 gpurun_out/r5ao/t_attn_vb1.log)"; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for n in vb0 vb1; do
    LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 300 python scripts/bench_mva.py > gpurun_out/r5ao/mva_${n}_r${round}.json 2> gpurun_out/r5ao/mva_${n}_r${round}.err || exit $?
    echo "$n r$round $(cat gpurun_out/r5ao/mva_${n}_r${round}.json)"
  done
done
