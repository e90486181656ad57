#!/bin/bash
# scratch iteration script for one gpurun call (overwritten per experiment)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out
RF_AMD_LIB=tools/ab/librf_amd_swz.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_compaction.py tests/test_gpu_fuzz.py > $O/gt_k.log 2>&1 || { tail -40 $O/gt_k.log; exit 1; }
tail -1 $O/gt_k.log
for r in 1 2 3; do for L in kbase swz; do
  RF_AMD_LIB=tools/ab/librf_amd_$L.so timeout -k 10 300 python bench.py --workload compaction --steps 5 --warmup 1 --no-cpu-baseline > $O/bk_$L.json 2> $O/bk_$L.err || { tail -20 $O/bk_$L.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bk_$L.json'));s=d['last_round_stages_ms'];print('$L', d['value'], d['ms_per_step'], d['verified'], s['cb_sort'], s['build_total'])"
done; done
for L in swzst; do
PT_LIB=tools/ab/librf_amd_$L.so PT_CHAIN=8 timeout -k 10 200 python tools/phase_times.py 1 64 1048575 > $O/pt1_chain8_$L.txt 2>&1 || exit 1
tail -13 $O/pt1_chain8_$L.txt
done
for L in kbase swz; do
  RF_AMD_LIB=tools/ab/librf_amd_$L.so timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $O/sqk_$L -o comp -- python3 bench.py --workload compaction --steps 2 --warmup 0 --no-cpu-baseline > $O/sqk_$L.log 2>&1 || { echo "sq $L failed"; exit 1; }
  python3 tools/sq_summary.py $O/sqk_$L/comp_counter_collection.csv > $O/sqk_$L.txt 2>&1; grep -i "cb_sort" $O/sqk_$L.txt | head -4
done
