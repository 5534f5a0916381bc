#!/bin/bash
# gpu_round.sh followed by the interleaved A/B of the variant libraries; stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_round.sh || exit $?
bash scripts/gpu_ab.sh
