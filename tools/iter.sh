#!/bin/bash
# scratch iteration script for one gpurun call (overwritten per experiment)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_compaction.py -k "ties or chain_rounds" > $O/gt_m6.log 2>&1 || { tail -40 $O/gt_m6.log; exit 1; }
tail -1 $O/gt_m6.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_shim.py tests/test_gpu_filter_test.py tests/test_gpu_parity.py > $O/gt_a.log 2>&1 || { tail -30 $O/gt_a.log; exit 1; }
tail -1 $O/gt_a.log
timeout -k 10 200 python tools/ab_step.py tools/ab/librf_amd_x3off.so tools/ab/librf_amd_x3on.so > $O/ab_x3.json 2>/dev/null || exit 1
cat $O/ab_x3.json
for m in 0 1; do
  RF_AMD_K6_MERGE=$m timeout -k 10 300 python bench.py --workload compaction --steps 5 --warmup 1 --no-cpu-baseline > $O/bc_m$m.json 2> $O/bc_m$m.err || { tail -20 $O/bc_m$m.err; exit 1; }
done
python -c "
import json
for m in (0,1):
    d=json.load(open('$O/bc_m%d.json'%m)); print(m, d['value'], d.get('ms_per_step'), d.get('verified'), d.get('kernels'))"
timeout -k 10 300 python tools/shim_latency.py > $O/sl_d1.json 2>/dev/null || exit 1
RF_SHIM_DIRECT=0 timeout -k 10 300 python tools/shim_latency.py > $O/sl_d0p1.json 2>/dev/null || exit 1
timeout -k 10 120 python tools/phase_times.py 2 > $O/pt2.txt 2>&1 || exit 1
timeout -k 10 120 python tools/phase_times.py 4 > $O/pt4.txt 2>&1 || exit 1
