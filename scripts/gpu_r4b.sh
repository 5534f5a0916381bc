#!/bin/bash
# Round-4 session B, most important first: (1) render parity tests on the one-wavefront backward (lib_bwdq); (2) one
# A/B round of the render variants (pool + cfg3 kernel times): lib_zf (current default), lib_bwdq, lib_wt
# (write-through hand-off stores), lib_sorth (sort keeps its histogram ranks), lib_bch (backward T (1 - alpha));
# (3) attention: bench_attn on lib_zf / lib_att1 / lib_att2 and the attention tests on lib_att2; (4) output hashes
# of the bitwise-equal variants; (5) a second A/B round; (6) the bwdq timelines.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V=$PWD/lgm_amd/_lib/variants
step() { echo "== $1 $(date +%s)"; }
ab() {  # $1 variant, $2 round
  LGM_AMD_LIB=$V/lib_$1.so timeout -k 10 150 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-attention --no-cfg4 --no-cfg5 --no-det > gpurun_out/ab_$1_r$2.json 2>/dev/null || return $?
  python -c "import json;b=json.load(open('gpurun_out/ab_$1_r$2.json'));c=b['cfg3_view_sharded'];print('$1 r$2', b['ms_per_step'], {k:v['avg_us'] for k,v in b['kernels'].items()}, 'cfg3', c['ms_per_step'], {k:v['avg_us'] for k,v in c['kernels'].items()})"
}
step tests_bwdq
LGM_AMD_LIB=$V/lib_bwdq.so timeout -k 10 420 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_render_parity_gpu.py tests/test_render_gpu.py tests/test_loss_gpu.py tests/test_training_gpu.py > gpurun_out/t_bwdq.log 2>&1
rc=$?; tail -3 gpurun_out/t_bwdq.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in zf bwdq wt sorth bch; do step "ab $v r1"; ab $v 1 || exit $?; done
for v in zf att1 att2; do
  step "attn $v"; LGM_AMD_LIB=$V/lib_$v.so timeout -k 10 200 python scripts/bench_attn.py --no-sdpa --iters 20 > gpurun_out/attn_$v.jsonl 2>/dev/null || exit $?
  python -c "
import json
for l in open('gpurun_out/attn_$v.jsonl'):
    r=json.loads(l); print('$v', r['level'], 'fwd %.0f TF fwdbwd %.0f TF' % (r['fwd_tflops'], r['fwdbwd_tflops']), {k: round(v, 3) for k, v in r['kernels_ms'].items()})"
done
step tests_att2
LGM_AMD_LIB=$V/lib_att2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/t_att2.log 2>&1
ra=$?; tail -3 gpurun_out/t_att2.log; [ $ra -eq 0 ] || [ $ra -eq 1 ] || exit $ra
for v in zf wt sorth; do step hash_$v; LGM_AMD_LIB=$V/lib_$v.so timeout -k 10 120 python scripts/render_hashes.py 2>/dev/null | tail -1 > gpurun_out/hash_$v.json || exit $?; cat gpurun_out/hash_$v.json; done
for v in zf bwdq wt sorth; do step "ab $v r2"; ab $v 2 || exit $?; done
step tl_bwdq
LGM_AMD_LIB=$V/lib_bwdq.so timeout -k 10 150 python scripts/diag_timeline.py 1 > gpurun_out/tl1_bwdq.log 2>&1 || exit $?
mv gpurun_out/timeline_B1.npz gpurun_out/timeline_B1_bwdq.npz
grep -v amdgpu.ids gpurun_out/tl1_bwdq.log
step tl_hw  # the in-tree library (default build, with the forward's hardware-placement stamps)
timeout -k 10 150 python scripts/diag_timeline.py 1 > gpurun_out/tl1_hw.log 2>&1 || exit $?
mv gpurun_out/timeline_B1.npz gpurun_out/timeline_B1_hw.npz
exit $rc
