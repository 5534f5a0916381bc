#!/bin/bash
# Round-4 session S: the single-scene timed loop after the pool (as in bench.py): 40 steps after 5 warmups,
# collector on / collected first / off, then 300 steps for reference.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for m in on collect off collect; do
  echo "== pool-first gc $m $(date +%s)"
  timeout -k 10 150 python scripts/diag_host.py --pool-first --steps 40 --warmup 5 --gc $m 2>/dev/null | tail -1 | tee -a gpurun_out/diag_host2.jsonl || exit $?
done
echo "== pool-first 300 steps $(date +%s)"
timeout -k 10 150 python scripts/diag_host.py --pool-first --steps 300 --warmup 5 --gc collect 2>/dev/null | tail -1 | tee -a gpurun_out/diag_host2.jsonl || exit $?
