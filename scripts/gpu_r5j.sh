#!/bin/bash
# Round-5 session J: host profile of the step that starts on an idle GPU (cProfile, scripts/diag_first_step_prof.py).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5j
timeout -k 10 300 python scripts/diag_first_step_prof.py > gpurun_out/r5j/prof.txt 2>&1 || exit $?
cat gpurun_out/r5j/prof.txt | grep -v "^$" | head -80
