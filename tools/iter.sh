#!/bin/bash
# scratch iteration script for one gpurun call (overwritten per experiment)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_compaction.py tests/test_gpu_fuzz.py > $O/gt_k.log 2>&1 || { tail -40 $O/gt_k.log; exit 1; }
tail -1 $O/gt_k.log
for r in 1 2; do for L in kbase knew; do
  RF_AMD_LIB=tools/ab/librf_amd_$L.so timeout -k 10 300 python bench.py --workload compaction --steps 5 --warmup 1 --no-cpu-baseline > $O/bk_$L.json 2> $O/bk_$L.err || { tail -20 $O/bk_$L.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bk_$L.json'));print('$L', d['value'], d['ms_per_step'], d['verified'], d['last_round_stages_ms'])"
done; done
PT_CHAIN=8 timeout -k 10 200 python tools/phase_times.py 1 64 1048575 > $O/pt1_chain8.txt 2>&1 || exit 1
tail -13 $O/pt1_chain8.txt
