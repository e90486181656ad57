#!/bin/bash
# One round's measurement evidence on the GPU box (run from the repo root via gpurun):
#   1. PMC passes FETCH_SIZE and WRITE_SIZE, separately (MI355X_MICROARCH.md HBM section),
#      summarised to per-launch HBM bytes per kernel;
#   2. rocprofv3 --kernel-trace --stats of the default bench command;
#   3. the bench lines (c2 with the CPU baseline, c3, c4, c5, routed, compaction) with roofline
#      traffic from (1), the compaction chain's kernel trace, the shim's per-call costs and the
#      reference's own kvstore driving the shim (tools/trunk_latency.py).
# usage: bash tools/profile_round.sh <tag> [a|b]   (outputs under gpurun_out/prof_<tag>/; a = PMC,
# traces and the C2-C5 bench lines, b = L2 counters, C3 trace/SQ, compaction, drop-in latencies;
# both when omitted -- two calls keep each under gpurun's limit)
set -o pipefail
TAG=${1:-r05}
PART=${2:-ab}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/prof_$TAG
mkdir -p $O
BENCH="bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e"
SQ="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU"
if [[ $PART == *a* ]]; then
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf -o c2 -- python3 $BENCH > $O/pf.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw -o c2 -- python3 $BENCH > $O/pw.log 2>&1 || { echo "pmc write failed"; exit 1; }
python3 profiles/pmc_summary.py $O/pf/c2_counter_collection.csv $O/pw/c2_counter_collection.csv $O/pmc_$TAG.json || exit 1
timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/sq -o c2 -- python3 $BENCH > $O/sq.log 2>&1 || { echo "pmc sq failed"; exit 1; }
python3 tools/sq_summary.py $O/sq/c2_counter_collection.csv > $O/sq_$TAG.txt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o c2 -- python3 $BENCH > $O/kt.log 2>&1 || { echo "kernel trace failed"; exit 1; }
timeout -k 10 400 python3 bench.py --pmc $O/pmc_$TAG.json > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench c2 failed"; exit 1; }
timeout -k 10 300 python3 bench.py --workload c3 --no-cpu-baseline --pmc none > $O/bench_c3.json 2> $O/bench_c3.err || { echo "bench c3 failed"; exit 1; }
timeout -k 10 300 python3 bench.py --workload c4 --no-cpu-baseline --pmc none > $O/bench_c4.json 2> $O/bench_c4.err || { echo "bench c4 failed"; exit 1; }
timeout -k 10 300 python3 bench.py --workload c5 --pmc none > $O/bench_c5.json 2> $O/bench_c5.err || { echo "bench c5 failed"; exit 1; }
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --routed-probe --pmc none > $O/bench_c2_routed.json 2> $O/bench_c2_routed.err || { echo "bench routed failed"; exit 1; }
fi
if [[ $PART == *b* ]]; then
# L2 behaviour of the probe (and every kernel) at C2 and C3: hits, misses, HBM read requests
TCC="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
timeout -s KILL 120 rocprofv3 --pmc $TCC --output-format csv -d $O/tcc2 -o c2 -- python3 $BENCH > $O/tcc2.log 2>&1 || { echo "pmc tcc c2 failed"; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc $TCC --output-format csv -d $O/tcc3 -o c3 -- python3 $BENCH --workload c3 > $O/tcc3.log 2>&1 || { echo "pmc tcc c3 failed"; exit 1; }
python3 tools/tcc_summary.py $O/tcc2/c2_counter_collection.csv $O/tcc3/c3_counter_collection.csv > $O/tcc_$TAG.txt || exit 1
# C3 (L2-resident line tables): kernel trace and SQ counters of the probe and the build
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt3 -o c3 -- python3 $BENCH --workload c3 > $O/kt3.log 2>&1 || { echo "c3 kernel trace failed"; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc $SQ --output-format csv -d $O/sq3 -o c3 -- python3 $BENCH --workload c3 > $O/sq3.log 2>&1 || { echo "pmc sq c3 failed"; exit 1; }
python3 tools/sq_summary.py $O/sq3/c3_counter_collection.csv > $O/sq_c3_$TAG.txt || exit 1
timeout -k 10 300 python3 bench.py --workload compaction --steps 5 --warmup 1 > $O/bench_compaction.json 2> $O/bench_compaction.err || { echo "bench compaction failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktc -o comp -- python3 bench.py --workload compaction --steps 2 --warmup 0 --no-cpu-baseline > $O/ktc.log 2>&1 || { echo "compaction kernel trace failed"; exit 1; }
# the drop-in's per-call costs beside the reference's routing_filter.c (tools/shim_latency.py)
timeout -k 10 600 python3 tools/shim_latency.py > $O/shim_latency_$TAG.json 2> $O/shim_latency.err || { echo "shim latency failed"; exit 1; }
timeout -k 10 300 python3 tools/trunk_latency.py > $O/trunk_latency_$TAG.json 2> $O/trunk_latency.err || { echo "trunk latency failed"; exit 1; }
fi
cat $O/bench_c2.json 2>/dev/null || true
