#!/bin/bash
# r05 call 40: GPU tests, default bench and compaction line with the K6 rework
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05d40
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1 || { echo "gpu tests failed"; tail -30 $O/gputest.txt; exit 1; }
tail -1 $O/gputest.txt
timeout -k 10 400 python3 bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench c2 failed"; tail $O/bench_c2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_c2.json').read().strip().splitlines()[-1]); print('c2', d['value'], d['ms_per_step'], d['kernels'], d['roofline']['frac'], d['verified'])" | cut -c1-800
timeout -k 10 300 python3 bench.py --workload compaction --steps 5 --warmup 1 > $O/bench_compaction.json 2> $O/bench_compaction.err || { echo "bench compaction failed"; tail $O/bench_compaction.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_compaction.json').read().strip().splitlines()[-1]); print('comp', d['value'], d['ms_per_step'], d['last_round_stages_ms'], d['verified'])"
