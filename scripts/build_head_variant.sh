#!/bin/bash
# Build the committed HEAD (or the given rev) as lgm_amd/_lib/variants/lib_a_head.so for an interleaved A/B
# against the working tree (scripts/gpu_ab.sh). Usage: scripts/build_head_variant.sh [rev]
set -e
REPO=$(cd "$(dirname "$0")/.." && pwd)
REV=${1:-HEAD}
TMP=$(mktemp -d /tmp/lgm_head.XXXXXX)
git -C "$REPO" worktree add -f "$TMP" "$REV" >/dev/null 2>&1
mkdir -p "$TMP/lgm_amd/_lib" "$REPO/lgm_amd/_lib/variants"
(cd "$TMP" && python -c "from lgm_amd import build as B; B.build(out='$REPO/lgm_amd/_lib/variants/lib_a_head.so')")
git -C "$REPO" worktree remove --force "$TMP"
echo "$REPO/lgm_amd/_lib/variants/lib_a_head.so"
