#!/bin/bash
# Round-4 session Q: host overhead of the single-scene step (scripts/diag_host.py), collector on / off / frozen.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for m in on off freeze on; do
  echo "== gc $m $(date +%s)"
  timeout -k 10 120 python scripts/diag_host.py --steps 300 --gc $m 2>/dev/null | tail -1 | tee -a gpurun_out/diag_host.jsonl || exit $?
done
