#!/bin/bash
# scratch iteration script for one gpurun call (overwritten per experiment)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py > $O/gt_p.log 2>&1 || { tail -30 $O/gt_p.log; exit 1; }
tail -1 $O/gt_p.log
timeout -k 10 200 python tools/ab_step.py tools/ab/librf_amd_pbase.so tools/ab/librf_amd_pnew.so > $O/ab_p.json 2>/dev/null || exit 1
cat $O/ab_p.json
for L in pbase pnew; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_BUSY_CYCLES --output-format csv -d $O/sq_$L -o p -- python3 tools/ab_step.py tools/ab/librf_amd_$L.so > $O/sq_$L.log 2>&1 || { echo "sq $L failed"; exit 1; }
  python3 tools/sq_summary.py $O/sq_$L/p_counter_collection.csv | grep -E "^probe" || true
done
