#!/bin/bash
# Round-5 session X: split-KV forward for grids that leave the chip idle (lib_split: this tree) against HEAD
# (lib_base): all attention GPU tests on split, then scripts/bench_attn.py and scripts/diag_cfg4.py per library,
# two interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5x
V=$PWD/lgm_amd/_lib/variants
LGM_AMD_LIB=$V/lib_split.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py -m gpu > gpurun_out/r5x/t_attn_split.log 2>&1
rc=$?; echo "split tests: $(tail -1 gpurun_out/r5x/t_attn_split.log)"; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for n in base split; do
    LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 300 python scripts/bench_attn.py --no-sdpa --iters 20 > gpurun_out/r5x/attn_${n}_r${round}.jsonl 2> gpurun_out/r5x/attn_${n}_r${round}.err || exit $?
    python -c "
import json
for l in open('gpurun_out/r5x/attn_${n}_r${round}.jsonl'):
    r=json.loads(l); print('$n r$round', r['level'], 'fwd %.0f TF fwdbwd %.0f TF' % (r['fwd_tflops'], r['fwdbwd_tflops']), {k: round(1e3*v, 1) for k, v in r['kernels_ms'].items()})"
    LGM_AMD_LIB=$V/lib_$n.so timeout -k 10 300 python scripts/diag_cfg4.py > gpurun_out/r5x/cfg4_${n}_r${round}.txt 2> gpurun_out/r5x/cfg4_${n}_r${round}.err || exit $?
    echo "$n r$round $(head -1 gpurun_out/r5x/cfg4_${n}_r${round}.txt)"
  done
done
