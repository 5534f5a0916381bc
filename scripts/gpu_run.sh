#!/bin/bash
# The one GPU session runner (replaces the per-session launchers of rounds 4-5). Runs the named steps in order on the
# gpurun box, each under its own time limit, and stops at the first failure (no retries).
#
#   bash scripts/gpu_run.sh STEP [STEP ...]        (results under $OUT, default gpurun_out/run)
#
# steps:
#   tests[=PYTEST_ARGS]  pytest -m gpu (default: the whole suite; e.g. tests=tests/test_attention.py, or
#                        "tests=tests/test_render_gpu.py -k needle")
#   smoke                __graft_entry__.smoke()
#   bench[=N]            bench.py with its defaults, N times (default 1), unprofiled, as the driver runs it
#   benchargs=ARGS       bench.py ARGS once (e.g. "benchargs=--steps 40 --only-pool")
#   prof                 rocprofv3 --kernel-trace --stats of the default bench + per-grid split, then one rocprofv3
#                        run per PMC pass of scripts/pmc_passes.txt (counters only with --kernel-trace)
#   trace=ARGS           rocprofv3 --kernel-trace --stats of bench.py ARGS, split per grid (no counters)
#   ab[=LIBS]            interleaved A/B of lgm_amd/_lib/variants/lib_*.so (render: bench kernel times + output hashes)
#   abattn               the same for the attention kernels (scripts/bench_attn.py)
#   abmva[=LIBS]         bench.py --only-attn per variant library (MVAttention level, attention, cfg4)
#   py=SCRIPT [ARGS]     python SCRIPT ARGS (a diagnostic under scripts/), output to $OUT/<script>.log
#   tracepy=SCRIPT [ARGS]  rocprofv3 --kernel-trace --stats of python SCRIPT ARGS, split per grid (every kernel the
#                        script launches, library GEMMs and torch's own included)
#   pmcpy=SCRIPT [ARGS]  one rocprofv3 counter run per line of $PASSES (default scripts/pmc_passes.txt) over python
#                        SCRIPT ARGS (e.g. scripts/probe_cfg2.py with PASSES=scripts/pmc_passes_cfg2.txt), summarised
#   abwgrad=NAMES        per variant library lib_NAME.so: the weight-gradient tests, then scripts/bench_wgrad.py in
#                        two interleaved rounds
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/run}
mkdir -p "$OUT"
export TMPDIR=/tmp

summ() {  # one-line summary of a bench JSON line
  python -c "
import json, sys
b = json.load(open(sys.argv[1])); c = b.get('cfg3_view_sharded') or {}
print(b['value'], b['ms_per_step'], {k: v['avg_us'] for k, v in b.get('kernels', {}).items()}, 'cfg3', c.get('ms_per_step'),
      {k: v['avg_us'] for k, v in c.get('kernels', {}).items()}, 'cfg2', (b.get('cfg2') or {}).get('ms_per_step'),
      'attn', (b.get('attention') or {}).get('tflops'), 'mva', (b.get('mva_level') or {}).get('fused_ms'),
      'cfg4', (b.get('cfg4') or {}).get('attention_core_tflops'), 'cfg5', (b.get('cfg5') or {}).get('render_side_ms'))" "$1"
}

for step in "$@"; do
  name=${step%%=*}; arg=""; [ "$name" != "$step" ] && arg=${step#*=}
  echo "== $step $(date +%s)"
  case $name in
    tests)
      [ -z "$arg" ] && arg=tests
      # shellcheck disable=SC2086
      timeout -k 10 1000 python -u -m pytest $arg -m gpu -v -rA --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
      rc=$?; echo "pytest_exit=$rc"; grep -E "FAILED|ERROR|passed|failed" "$OUT/gpu_tests.log" | tail -12
      [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
      rc=$?; echo "smoke_exit=$rc"; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      for r in $(seq 1 "${arg:-1}"); do
        timeout -k 10 400 python bench.py > "$OUT/bench_plain$r.json" 2> "$OUT/bench_plain$r.err" || exit $?
        summ "$OUT/bench_plain$r.json"
      done ;;
    benchargs)
      # shellcheck disable=SC2086
      timeout -k 10 400 python bench.py $arg > "$OUT/bench_args.json" 2> "$OUT/bench_args.err" || exit $?
      summ "$OUT/bench_args.json" 2>/dev/null || python -c "import json,sys;b=json.load(open(sys.argv[1]));print({k:(v if not isinstance(v,dict) else {kk:vv for kk,vv in v.items() if kk!=\"timed_loop\"}) for k,v in b.items()})" "$OUT/bench_args.json" ;;
    prof)
      mkdir -p "$OUT/prof" "$OUT/pmc"
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py > "$OUT/prof/bench.json" 2> "$OUT/prof/bench.err"
      rc=$?; echo "stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
      python scripts/kernel_stats_by_grid.py "$OUT/prof/run_kernel_trace.csv" > "$OUT/prof/kernel_stats_by_grid.txt"
      summ "$OUT/prof/bench.json"
      i=0
      while read -r line; do
        [ -z "$line" ] && continue
        i=$((i+1))
        timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $line -d "$OUT/pmc/p$i" -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --only-pool --no-cpu-baseline > "$OUT/pmc/p$i.log" 2>&1
        rc=$?; echo "pass $i ($line) rc=$rc"; [ $rc -eq 0 ] || exit $rc
      done < scripts/pmc_passes.txt
      python scripts/pmc_summary.py "$OUT/pmc" --json "$OUT/pmc_latest.json" > "$OUT/pmc_summary.txt"; echo "pmc summary rc=$?" ;;
    trace)  # rocprofv3 kernel trace + stats of bench.py ARGS (no counters), split per grid
      mkdir -p "$OUT/trace"
      # shellcheck disable=SC2086
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python bench.py $arg > "$OUT/trace/bench.json" 2> "$OUT/trace/bench.err"
      rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
      python scripts/kernel_stats_by_grid.py "$OUT/trace/run_kernel_trace.csv" > "$OUT/trace/kernel_stats_by_grid.txt"
      head -40 "$OUT/trace/kernel_stats_by_grid.txt" ;;
    ab)
      OUTAB="$OUT/ab" AB_LIBS="$arg" bash scripts/gpu_ab.sh || exit $? ;;
    abattn)
      OUTAB="$OUT/ab" bash scripts/gpu_ab_attn.sh || exit $? ;;
    abmva)
      OUTAB="$OUT/ab" AB_LIBS="$arg" bash scripts/gpu_ab_mva.sh || exit $? ;;
    py)
      # shellcheck disable=SC2086
      set -- $arg; s=$1; shift
      timeout -k 10 600 python -u "$s" "$@" > "$OUT/$(basename "$s" .py).log" 2>&1
      rc=$?; echo "$s rc=$rc"; tail -5 "$OUT/$(basename "$s" .py).log"; [ $rc -eq 0 ] || exit $rc ;;
    tracepy)
      mkdir -p "$OUT/tracepy"
      # shellcheck disable=SC2086
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/tracepy" -o run --output-format csv -- python $arg > "$OUT/tracepy/run.log" 2>&1
      rc=$?; echo "tracepy rc=$rc"; [ $rc -eq 0 ] || exit $rc
      python scripts/kernel_stats_by_grid.py "$OUT/tracepy/run_kernel_trace.csv" > "$OUT/tracepy/kernel_stats_by_grid.txt"
      head -30 "$OUT/tracepy/kernel_stats_by_grid.txt" ;;
    pmcpy)
      mkdir -p "$OUT/pmcpy"
      i=0
      while read -r line; do
        [ -z "$line" ] && continue
        i=$((i+1))
        # shellcheck disable=SC2086
        timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $line -d "$OUT/pmcpy/p$i" -o run --output-format csv -- python $arg > "$OUT/pmcpy/p$i.log" 2>&1
        rc=$?; echo "pass $i ($line) rc=$rc"; [ $rc -eq 0 ] || exit $rc
      done < "${PASSES:-scripts/pmc_passes.txt}"
      python scripts/pmc_summary.py "$OUT/pmcpy" > "$OUT/pmcpy/summary.txt"; echo "pmc summary rc=$?" ;;
    abwgrad)
      mkdir -p "$OUT/wgab"
      for v in $arg; do
        LGM_AMD_LIB=$PWD/lgm_amd/_lib/variants/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_wgrad.py -m gpu -q --timeout 120 --timeout-method thread > "$OUT/wgab/t_$v.log" 2>&1
        rc=$?; echo "$v tests: $(tail -1 "$OUT/wgab/t_$v.log")"; [ $rc -eq 0 ] || exit $rc
      done
      for r in 1 2; do for v in $arg; do
        LGM_AMD_LIB=$PWD/lgm_amd/_lib/variants/lib_$v.so timeout -k 10 120 python scripts/bench_wgrad.py > "$OUT/wgab/${v}_r$r.jsonl" 2>&1 || exit $?
        echo "$v r$r"; grep '^{' "$OUT/wgab/${v}_r$r.jsonl"
      done; done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
