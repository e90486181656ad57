#!/bin/bash
# r05 call 42: SQ counters of the C2 step with the reworked K6 (VALU, LDS, conflicts per kernel)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05d42
mkdir -p $O
BENCH="bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e"
SQ="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU"
timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/sq -o c2 -- python3 $BENCH > $O/sq.log 2>&1 || { echo "pmc sq failed"; exit 1; }
python3 tools/sq_summary.py $O/sq/c2_counter_collection.csv > $O/sq_end.txt || exit 1
cat $O/sq_end.txt
