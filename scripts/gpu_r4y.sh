#!/bin/bash
# Round-4 session Y: the backward's LDS bank layout -- lib_mst (session X: moment stores on distinct banks) and
# lib_swz (that plus the w / u image's columns 4..11 swizzled for the batch reads) vs lib_base: hashes, render tests
# on lib_swz, LDS bank-conflict counters of the pool for all three, three base / swz A/B rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmcx
export TMPDIR=/tmp
V=$PWD/lgm_amd/_lib/variants
VARS="base swz"
step() { echo "== $1 $(date +%s)"; }
ab() {  # $1 variant, $2 round
  LGM_AMD_LIB=$V/lib_$1.so timeout -k 10 150 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-attention --no-cfg4 --no-cfg5 --no-det > gpurun_out/ab_$1_r$2.json 2>/dev/null || return $?
  python -c "import json;b=json.load(open('gpurun_out/ab_$1_r$2.json'));c=b['cfg3_view_sharded'];print('$1 r$2', b['ms_per_step'], {k:v['avg_us'] for k,v in b['kernels'].items()}, 'cfg3', c['ms_per_step'], c['step_spread']['median_ms'], {k:v['avg_us'] for k,v in c['kernels'].items()})"
}
for v in $VARS; do step hash_$v; LGM_AMD_LIB=$V/lib_$v.so timeout -k 10 120 python scripts/render_hashes.py 2>/dev/null | tail -1 > gpurun_out/hash_$v.json || exit $?; cat gpurun_out/hash_$v.json; done
step tests_swz
LGM_AMD_LIB=$V/lib_swz.so timeout -k 10 420 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_render_parity_gpu.py tests/test_render_gpu.py tests/test_loss_gpu.py tests/test_training_gpu.py > gpurun_out/t_swz.log 2>&1
rc=$?; tail -2 gpurun_out/t_swz.log; [ $rc -eq 0 ] || exit $rc
for v in base mst swz; do
  step "pmc $v"
  LGM_AMD_LIB=$V/lib_$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d gpurun_out/pmcx/$v -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --only-pool --no-cpu-baseline > gpurun_out/pmcx/$v.log 2>&1 || exit $?
  python - <<PY
import csv, glob, collections, re
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob('gpurun_out/pmcx/$v/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        mm = re.search(r'(k_[a-z_]+)', r['Kernel_Name'])
        if not mm: continue
        k = mm.group(1)
        acc[k][r['Counter_Name']] += float(r['Counter_Value'])
        if r['Counter_Name'] == 'SQ_LDS_IDX_ACTIVE': n[k] += 1
for k in ('k_render_bwd', 'k_render_fwd', 'k_bin', 'k_sort'):
    a = acc[k]
    if a: print('$v', k, 'conflict/active %.4f' % (a['SQ_LDS_BANK_CONFLICT'] / max(a['SQ_LDS_IDX_ACTIVE'], 1)), 'per launch conflict %.3e' % (a['SQ_LDS_BANK_CONFLICT'] / max(n[k], 1)))
PY
done
for r in 1 2 3; do for v in $VARS; do step "ab $v r$r"; ab $v $r || exit $?; done; done
