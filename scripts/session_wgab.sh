# A/B of weight-gradient variant libraries (scripts/bench_wgrad.py per library, 2 rounds), after the wgrad tests on each
cd $GRAFT_REPO_ROOT; OUT=${OUT:-gpurun_out/wgab}; mkdir -p $OUT
for v in $WG_LIBS; do
  LGM_AMD_LIB=$GRAFT_REPO_ROOT/lgm_amd/_lib/variants/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_wgrad.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/t_$v.log 2>&1
  rc=$?; echo "$v tests: $(tail -1 $OUT/t_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do for v in $WG_LIBS; do
  LGM_AMD_LIB=$GRAFT_REPO_ROOT/lgm_amd/_lib/variants/lib_$v.so timeout -k 10 120 python scripts/bench_wgrad.py > $OUT/${v}_r$r.jsonl 2>&1 || exit $?
  echo "$v r$r"; grep '^{' $OUT/${v}_r$r.jsonl
done; done
