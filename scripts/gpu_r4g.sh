#!/bin/bash
# Round-4 session H: backward LDS bank conflicts -- lib_junk (dead moment-MFMA results to per-lane junk words),
# lib_ls71 (moment-slot row stride 71: the flush's (entry, partial) reads over distinct banks), lib_ls71junk (both)
# against lib_base: hashes, render tests on lib_ls71junk, three A/B rounds, then one PMC pass (LDS counters) per arm.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmch
export TMPDIR=/tmp
V=$PWD/lgm_amd/_lib/variants
step() { echo "== $1 $(date +%s)"; }
ab() {  # $1 variant, $2 round
  LGM_AMD_LIB=$V/lib_$1.so timeout -k 10 150 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-attention --no-cfg4 --no-cfg5 --no-det > gpurun_out/ab_$1_r$2.json 2>/dev/null || return $?
  python -c "import json;b=json.load(open('gpurun_out/ab_$1_r$2.json'));c=b['cfg3_view_sharded'];print('$1 r$2', b['ms_per_step'], {k:v['avg_us'] for k,v in b['kernels'].items()}, 'cfg3', c['ms_per_step'], c['step_spread']['median_ms'], {k:v['avg_us'] for k,v in c['kernels'].items()})"
}
for v in base junk ls71 ls71junk hist4; do step hash_$v; LGM_AMD_LIB=$V/lib_$v.so timeout -k 10 120 python scripts/render_hashes.py 2>/dev/null | tail -1 > gpurun_out/hash_$v.json || exit $?; cat gpurun_out/hash_$v.json; done
rc=0
for v in ls71junk hist4; do
  step tests_$v
  LGM_AMD_LIB=$V/lib_$v.so timeout -k 10 420 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_render_parity_gpu.py tests/test_render_gpu.py tests/test_loss_gpu.py > gpurun_out/t_$v.log 2>&1
  r=$?; tail -2 gpurun_out/t_$v.log; [ $r -eq 0 ] || [ $r -eq 1 ] || exit $r; rc=$((rc | r))
done
for r in 1 2 3; do for v in base junk ls71 ls71junk hist4; do step "ab $v r$r"; ab $v $r || exit $?; done; done
for v in base ls71junk; do
  step pmc_$v
  LGM_AMD_LIB=$V/lib_$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS -d gpurun_out/pmch/$v/p1 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --only-pool --no-cpu-baseline > gpurun_out/pmch/$v.log 2>&1 || exit $?
done
python scripts/pmc_summary.py gpurun_out/pmch/base > gpurun_out/pmch/base.txt 2>&1; python scripts/pmc_summary.py gpurun_out/pmch/ls71junk > gpurun_out/pmch/ls71junk.txt 2>&1
exit $rc
