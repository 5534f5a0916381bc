#!/bin/bash
# Round-4 session A: whole-step timelines (B = 1 and the pool), a short bench, output hashes of the current library and
# of the pruned variant (must match), and the new GPU tests. Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() { echo "== $1"; }
step tl1; timeout -k 10 150 python scripts/diag_timeline.py 1 > gpurun_out/tl1.log 2>&1 || exit $?
step tl8; timeout -k 10 150 python scripts/diag_timeline.py 8 > gpurun_out/tl8.log 2>&1 || exit $?
step bench; timeout -k 10 200 python bench.py --steps 40 --warmup 10 --no-cpu-baseline --no-attention --no-cfg4 --no-cfg5 > gpurun_out/bench_head.json 2> gpurun_out/bench_head.err || exit $?
step hash; timeout -k 10 120 python scripts/render_hashes.py > gpurun_out/hash_head.json 2>&1 || exit $?
step hash_pruned; LGM_AMD_LIB=$PWD/lgm_amd/_lib/variants/lib_pruned.so timeout -k 10 120 python scripts/render_hashes.py > gpurun_out/hash_pruned.json 2>&1 || exit $?
step hash_zf; LGM_AMD_LIB=$PWD/lgm_amd/_lib/variants/lib_zf.so timeout -k 10 120 python scripts/render_hashes.py > gpurun_out/hash_zf.json 2>&1 || exit $?
for r in 1 2; do for v in pruned zf fch bch; do
  step "ab $v r$r"; LGM_AMD_LIB=$PWD/lgm_amd/_lib/variants/lib_$v.so timeout -k 10 150 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-attention --no-cfg4 --no-cfg5 --no-det > gpurun_out/ab_${v}_r$r.json 2>/dev/null || exit $?
  python -c "import json;b=json.load(open('gpurun_out/ab_${v}_r$r.json'));c=b['cfg3_view_sharded'];print('$v r$r', b['ms_per_step'], {k:v['avg_us'] for k,v in b['kernels'].items()}, 'cfg3', c['ms_per_step'], {k:v['avg_us'] for k,v in c['kernels'].items()})"
done; done
step hash_fch; LGM_AMD_LIB=$PWD/lgm_amd/_lib/variants/lib_fch.so timeout -k 10 120 python scripts/render_hashes.py > gpurun_out/hash_fch.json 2>&1 || exit $?
step tests; timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cameras_gpu.py tests/test_render_gpu.py tests/test_dist_gpu.py tests/test_attention.py -k "needle or orbit or device_cameras or accumulation or c512 or c1024" > gpurun_out/t1.log 2>&1
rc=$?
cat gpurun_out/tl1.log gpurun_out/tl8.log gpurun_out/hash_head.json gpurun_out/hash_pruned.json gpurun_out/hash_zf.json gpurun_out/hash_fch.json
grep -E "passed|failed|fancy|visible|Error" gpurun_out/t1.log
exit $rc
