#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
python -m lgm_amd.build > gpurun_out/build.log 2>&1 || { echo "build failed"; exit 1; }
timeout -k 10 120 python scripts/diag_counters.py > gpurun_out/counters.log 2>&1
echo "exit=$?"
