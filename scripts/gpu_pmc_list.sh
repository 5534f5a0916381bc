#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1
echo "exit=$?"
