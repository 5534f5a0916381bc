#!/bin/bash
# Float-atomic gradient spread at cfg4 512^2 (scripts/diag_float_spread.py): R float runs against the deterministic
# gradients; the arrays of the deterministic, worst and best float runs are kept for an fp64-oracle comparison.
# Variant libraries under lgm_amd/_lib/variants/ (if any) run the same with one float run each.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python scripts/diag_float_spread.py ${1:-8} > gpurun_out/spread_default.log 2>&1; rc=$?; echo "rc=$rc"
grep -v amdgpu.ids gpurun_out/spread_default.log | tail -10 | cut -c1-300
[ $rc -eq 0 ] || exit $rc
for lib in lgm_amd/_lib/variants/lib_*.so; do
  [ -e "$lib" ] || continue
  n=$(basename $lib .so)
  LGM_AMD_LIB=$PWD/$lib timeout -k 10 300 python scripts/diag_float_spread.py 1 _$n > gpurun_out/spread_$n.log 2>&1; rc=$?; echo "$n rc=$rc"
  grep -v amdgpu.ids gpurun_out/spread_$n.log | tail -2 | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
done
exit 0
