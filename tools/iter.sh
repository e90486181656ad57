#!/bin/bash
# r06 call 4: the lookup-server tests (ADVICE r5 dead-server test) and the two-stack latency tool
# run to its natural exit (no --fast-exit)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_server.py > $O/t_server.log 2>&1 || { echo "server tests failed"; tail -30 $O/t_server.log; exit 1; }
tail -3 $O/t_server.log
timeout -k 10 600 python3 tools/shim_latency.py > $O/shim_latency.json 2> $O/shim_latency.err
rc=$?
echo "shim_latency rc=$rc"
tail -5 $O/shim_latency.err
exit $rc
