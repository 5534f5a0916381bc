#!/bin/bash
# Round-5 session AA: XCD balance of one cfg3 scene's forward tiles and backward items (scripts/diag_xcd.py).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5aa
timeout -k 10 300 python scripts/diag_xcd.py > gpurun_out/r5aa/xcd.json 2> gpurun_out/r5aa/xcd.err
rc=$?; python -c "
import json
d=json.load(open('gpurun_out/r5aa/xcd.json'))
for k, v in d.items():
    print(k, 'fwd span', v['fwd_span_us'], 'bwd span', v['bwd_span_us'])
    for kk, vv in v.items():
        if isinstance(vv, dict): print('  ', kk, vv)
" ; exit $rc
