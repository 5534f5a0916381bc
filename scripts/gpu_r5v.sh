#!/bin/bash
# Round-5 session V: where cfg4's attention pass spends its time (scripts/diag_cfg4.py).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5v
timeout -k 10 300 python scripts/diag_cfg4.py > gpurun_out/r5v/diag_cfg4.txt 2> gpurun_out/r5v/diag_cfg4.err
rc=$?; head -c 6000 gpurun_out/r5v/diag_cfg4.txt; exit $rc
