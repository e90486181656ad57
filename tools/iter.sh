#!/bin/bash
# r06 call 15: probe lines v2 at the old table sizes (RF_AMD_LINE_SIGMA=5: 8 lines per index at
# C2 and C3, no overflow walks) -- the decode's own cost
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06o
mkdir -p $O
for W in c2 c3; do
  RF_AMD_LINE_SIGMA=5 timeout -k 10 300 python3 bench.py --workload $W --no-cpu-baseline --no-e2e --pmc none > $O/bench_${W}_s5.json 2> $O/bench_${W}_s5.err || { echo "bench $W failed"; tail -5 $O/bench_${W}_s5.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_${W}_s5.json')); print('$W sigma5', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('probe_floor'))"
done
