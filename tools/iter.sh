#!/bin/bash
# r06 session 2, call 13: per-thread burst detection (batch path after 64 first calls with no DONE); drop-in latencies
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06s2m
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_server.py tests/test_gpu_shim.py tests/test_gpu_trunk.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
AD_REPS=9 timeout -k 10 200 python3 -u tools/async_driven.py > $O/ad_$i.json 2> $O/ad_$i.err || { echo ad failed; tail -20 $O/ad_$i.err; exit 1; }
echo "run $i: $(cat $O/ad_$i.json)"
done
timeout -k 10 400 python3 tools/shim_latency.py > $O/shim_latency.json 2> $O/shim_latency.err || { echo shim latency failed; tail -5 $O/shim_latency.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/shim_latency.json'))
for s in ('shim','reference'): print(s, {k: d[s].get(k) for k in ('lookup_one_ms','lookup_async_8192_ms','lookup_async_8192_detail','async_driven_8192_ms','async_8192_512f_ms')})"
timeout -k 10 300 python3 tools/trunk_latency.py > $O/trunk_latency.json 2> $O/trunk_latency.err || { echo trunk latency failed; tail -5 $O/trunk_latency.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/trunk_latency.json'))
for s in ('shim','reference'): print(s, {k: d[s]['second'].get(k) for k in ('lookup_hit_us','lookup_async64_hit_us','lookup_miss_us','lookup_async64_miss_us')})"
