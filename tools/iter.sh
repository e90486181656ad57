#!/bin/bash
# r05 call 27: reaper A/B (per-slot tickets vs served head) on one box; then the exit abort's backtrace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05d27
mkdir -p $O
ulimit -c 0
for v in 1 0 1 0; do
  RF_AMD_REAP_TICKETS=$v timeout -k 10 600 python3 tools/shim_latency.py --fast-exit > $O/sl_$v.json 2> $O/sl_$v.err || { echo "shim_latency $v failed"; tail -5 $O/sl_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/sl_$v.json'))['shim']; print('tickets=$v', d['async_driven_8192_ms'], d['async_driven_breakdown'], d['lookup_async_8192_ms'], d['lookup_one_ms'])"
done
RFR_ABORT_BT=1 timeout -k 10 600 python3 tools/shim_latency.py > $O/sl_bt.json 2> $O/sl_bt.err; echo "bt run rc $?"
grep -v "UserWarning\|setattr\|return self._float" $O/sl_bt.err | tail -40
