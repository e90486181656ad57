#!/bin/bash
# r05 call 8: full GPU suite on the round-5 changes; ping-pong; kvstore insert breakdown
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05d8
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/gputest.log 2>&1 || { echo "gpu tests failed"; tail -60 $O/gputest.log; exit 1; }
tail -3 $O/gputest.log
timeout -k 10 60 ./tools/pingpong > $O/pingpong.txt 2>&1 || { echo "pingpong failed"; cat $O/pingpong.txt; exit 1; }
cat $O/pingpong.txt
timeout -k 10 400 python3 tools/trunk_latency.py > $O/trunk_latency.json 2> $O/trunk_latency.err || { echo "trunk latency failed"; tail $O/trunk_latency.err; exit 1; }
cat $O/trunk_latency.json
