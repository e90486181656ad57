#!/bin/bash
# scratch iteration script for one gpurun call (overwritten per experiment)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
O=gpurun_out
for r in 1 2; do
for t in 1; do
RF_SHIM_BATCH_THREADS=$t timeout -k 10 300 python tools/shim_latency.py > $O/sl_t$t.json 2>/dev/null || exit 1
python -c "
import json; d=json.load(open('$O/sl_t$t.json'))['shim']; print($t, {k:d[k] for k in ('add_fresh_ms','mt_adds_8x_ms','lookup_one_ms','lookup_batch_8192_ms','lookup_async_8192_ms','async_driven_8192_ms','async_8192_512f_ms')})"
done
done
