#!/bin/bash
# scratch iteration script for one gpurun call (overwritten per experiment)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
O=gpurun_out
RF_AMD_LIB=tools/ab/librf_amd_uw.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_compaction.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py > $O/gt_k.log 2>&1 || { tail -40 $O/gt_k.log; exit 1; }
tail -1 $O/gt_k.log
timeout -k 10 400 python3 tools/ab_probe2.py tools/ab/librf_amd_base.so tools/ab/librf_amd_uw.so > $O/ab_uw.json 2> $O/ab_uw.err || { tail -20 $O/ab_uw.err; exit 1; }
cat $O/ab_uw.json; echo
for r in 1 2 3; do for L in base uw; do
  RF_AMD_LIB=tools/ab/librf_amd_$L.so timeout -k 10 300 python bench.py --workload compaction --steps 5 --warmup 1 --no-cpu-baseline > $O/bk_$L.json 2> $O/bk_$L.err || { tail -20 $O/bk_$L.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bk_$L.json'));s=d['last_round_stages_ms'];print('$L', d['value'], d['ms_per_step'], d['verified'], s['cb_sort'], s['build_total'])"
done; done
