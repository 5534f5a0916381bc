#!/bin/bash
# Round evidence: build + GPU tests + counters + bench + rocprofv3 kernel stats (gpu_round.sh), then the PMC passes
# (gpu_pmc.sh) summarised to gpurun_out/pmc_latest.json. Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_round.sh || exit $?
bash scripts/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc.log; exit 1; }
python scripts/pmc_summary.py gpurun_out/pmc --json gpurun_out/pmc_latest.json > gpurun_out/pmc_summary.txt
echo "pmc ok"
