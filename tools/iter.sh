#!/bin/bash
# scratch iteration script for one gpurun call (overwritten per experiment)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_server.py tests/test_gpu_shim.py tests/test_gpu_trunk.py tests/test_gpu_filter_test.py > $O/gt_d.log 2>&1 || { tail -40 $O/gt_d.log; exit 1; }
tail -1 $O/gt_d.log
timeout -k 10 300 python tools/shim_latency.py > $O/sl_f.json 2>/dev/null || exit 1
python -c "
import json; d=json.load(open('$O/sl_f.json'))['shim']; print({k:d[k] for k in ('add_fresh_ms','add_incremental_ms','mt_adds_8x_ms','lookup_one_ms','lookup_batch_8192_ms','lookup_async_8192_ms','async_driven_8192_ms','async_8192_512f_ms')}); print(d['async_driven_breakdown'])"
timeout -k 10 300 python tools/trunk_latency.py > $O/trunk_f.json 2>/dev/null || exit 1
cat $O/trunk_f.json
