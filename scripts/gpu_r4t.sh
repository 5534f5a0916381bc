#!/bin/bash
# Round-4 session T: slot-mode bucket stride capped at 16k / 8k entries (lib_s16k, lib_s8k: a 1.2 GB -> 197 / 98 MB
# pair span for one scene, 9.8 GB -> 1.6 / 0.8 GB for the pool) vs N (lib_base): does the sparse span cost
# translation misses? The caps are only safe below the workloads' largest tile list (printed first).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V=$PWD/lgm_amd/_lib/variants
step() { echo "== $1 $(date +%s)"; }
ab() {  # $1 variant, $2 round
  LGM_AMD_LIB=$V/lib_$1.so timeout -k 10 150 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-attention --no-cfg4 --no-cfg5 --no-det > gpurun_out/ab_$1_r$2.json 2>/dev/null || return $?
  python -c "import json;b=json.load(open('gpurun_out/ab_$1_r$2.json'));c=b['cfg3_view_sharded'];print('$1 r$2', b['ms_per_step'], {k:v['avg_us'] for k,v in b['kernels'].items()}, 'cfg3', c['ms_per_step'], c['step_spread']['median_ms'], {k:v['avg_us'] for k,v in c['kernels'].items()})"
}
step maxcount
LGM_AMD_LIB=$V/lib_base.so timeout -k 10 120 python scripts/max_tile_count.py 2>/dev/null | tee gpurun_out/maxcount.txt || exit $?
mx=$(awk '{print $3}' gpurun_out/maxcount.txt | sort -n | tail -1)
VARS="base s16k"
[ "$mx" -lt 8192 ] && VARS="base s16k s8k"
[ "$mx" -lt 16384 ] || { echo "largest list $mx >= 16384: no capped run"; exit 0; }
for v in $VARS; do step hash_$v; LGM_AMD_LIB=$V/lib_$v.so timeout -k 10 120 python scripts/render_hashes.py 2>/dev/null | tail -1 > gpurun_out/hash_$v.json || exit $?; cat gpurun_out/hash_$v.json; done
for r in 1 2 3; do for v in $VARS; do step "ab $v r$r"; ab $v $r || exit $?; done; done
