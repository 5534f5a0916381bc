#!/bin/bash
# Round-5 session AN: k_mva_out with vector accesses, all loads in flight (k_mva_out_v, LGM_MVA_VEC=1: lib_vo1)
# against the scalar-width k_mva_out (lib_vo0): attention GPU tests on vo1, then scripts/bench_mva.py and
# scripts/diag_cfg4.py per library, two rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5an
V=$PWD/lgm_amd/_lib/variants_attn
LGM_AMD_LIB=$V/lib_vo1.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/r5an/t_attn_vo1.log 2>&1
rc=$?; echo "vo1 tests: $(tail -1 gpurun_out/r5an/t_attn_vo1.log)"; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for n in vo0 vo1; do
    LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 300 python scripts/bench_mva.py > gpurun_out/r5an/mva_${n}_r${round}.json 2> gpurun_out/r5an/mva_${n}_r${round}.err || exit $?
    echo "$n r$round $(cat gpurun_out/r5an/mva_${n}_r${round}.json)"
    LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 300 python scripts/diag_cfg4.py > gpurun_out/r5an/cfg4_${n}_r${round}.json 2> gpurun_out/r5an/cfg4_${n}_r${round}.err || exit $?
    echo "$n r$round cfg4 $(head -c 400 gpurun_out/r5an/cfg4_${n}_r${round}.json)"
  done
done
