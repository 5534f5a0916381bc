#!/bin/bash
# DMA lane-stride probe (lgm_amd/_lib/dma_probe, built on the host) followed by the variant A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 60 ./lgm_amd/_lib/dma_probe; rc=$?; echo "probe_exit=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/gpu_ab.sh
