#!/bin/bash
# r05 call 25: reaper polls the server's served-head word; K4m uniq by wave sums
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05d25
mkdir -p $O
ulimit -c 0
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_server.py tests/test_gpu_shim.py tests/test_gpu_trunk.py tests/test_gpu_compaction.py tests/test_gpu_fuzz.py > $O/t.log 2>&1 || { echo "tests failed"; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 600 python3 tools/shim_latency.py > $O/shim_latency.json 2> $O/shim_latency.err; echo "shim_latency rc $?"
python3 -c "import json; d=json.load(open('$O/shim_latency.json'))['shim']; print({k: d[k] for k in ('lookup_one_ms','lookup_async_8192_ms','async_driven_8192_ms','async_driven_breakdown','async_8192_512f_ms')})"
