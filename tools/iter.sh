#!/bin/bash
# r06 call 22: pool default raised: stall tool + compaction bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06v
mkdir -p $O
timeout -k 10 300 python3 -u tools/chain_stall.py > $O/stall.txt 2>&1 || { echo stall failed; tail -5 $O/stall.txt; exit 1; }
tail -3 $O/stall.txt
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --workload compaction --no-cpu-baseline --pmc none > $O/bc_$i.json 2> $O/bc_$i.err || { echo bench failed; tail -5 $O/bc_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bc_$i.json')); print($i, d['value'], d['ms_per_step'], d['round_wall_ms'], d['round_build_ms'], d['with_readback']['round_wall_ms'], d['verified'])"
done
