#!/bin/bash
# Round-4 session U: does an idle GPU before the timed loop slow its first steps (clock ramp)? 400 single-scene
# steps after 0 / 100 / 300 ms of idle, GPU time per step averaged over each 20 steps.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for ms in 0 100 300 0 100; do
  echo "== idle $ms $(date +%s)"
  timeout -k 10 150 python scripts/diag_host.py --steps 400 --warmup 20 --idle-ms $ms 2>/dev/null | tail -1 | tee -a gpurun_out/diag_idle.jsonl || exit $?
done
