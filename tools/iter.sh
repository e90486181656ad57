#!/bin/bash
# r05 call 44: PMC HBM traffic (FETCH_SIZE, WRITE_SIZE passes) of the final round-5 code
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05d44
mkdir -p $O
BENCH="bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf -o c2 -- python3 $BENCH > $O/pf.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw -o c2 -- python3 $BENCH > $O/pw.log 2>&1 || { echo "pmc write failed"; exit 1; }
python3 profiles/pmc_summary.py $O/pf/c2_counter_collection.csv $O/pw/c2_counter_collection.csv $O/pmc_end.json || exit 1
python3 -c "import json; d=json.load(open('$O/pmc_end.json')); print(json.dumps(d['per_launch_hbm_bytes']))"
