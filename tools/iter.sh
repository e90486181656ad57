#!/bin/bash
# r05 call 31: C3/C4/C5 bench lines with the final probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05d31
mkdir -p $O
for w in c3 c4; do
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline --pmc none > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail $O/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$w.json').read().strip().splitlines()[-1]); print('$w', d['value'], d['kernels']['probe']['ms'], d['probe_floor']['floor_ms'], d['probe_floor']['probe_over_floor'], d['roofline']['frac'], d['verified'])"
done
