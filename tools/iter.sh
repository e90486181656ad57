#!/bin/bash
# r05 call 30: K4m with K4M_PER buckets per workgroup (next bucket's new entries prefetched): tests, A/B 1/2/4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05d30
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_compaction.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py > $O/t.log 2>&1 || { echo "tests failed"; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 600 python3 tools/ab_chain.py tools/ab/librf_amd_per1.so tools/ab/librf_amd_per2.so splinterdb_amd/librf_amd.so > $O/ab_chain.json 2> $O/ab_chain.err || { echo "ab failed"; tail $O/ab_chain.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/ab_chain.json')); print(d['identical'], {k: (v['cb_sort'], v['build_total']) for k, v in d['stages_ms_median'].items()})"
