#!/bin/bash
# r06 call 6: the two-stack latency tool to its natural exit after the harness buffer fix, and
# the drop-in's GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
RFR_ABORT_BT=1 timeout -k 10 600 python3 tools/shim_latency.py > $O/shim_latency.json 2> $O/shim_latency.err
rc=$?
echo "shim_latency rc=$rc"
grep -v UserWarning $O/shim_latency.err | grep -v "setattr\|return self" | tail -30
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_shim.py tests/test_gpu_trunk.py > $O/t_shim.log 2>&1; echo "shim tests rc=$?"; tail -5 $O/t_shim.log
