#!/bin/bash
# r05 call 22: K4m fallback on a full grid (compaction chain), exit-abort bisect mode 9 last
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05d22
mkdir -p $O
ulimit -c 0
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_compaction.py tests/test_gpu_fuzz.py > $O/t.log 2>&1 || { echo "tests failed"; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python3 bench.py --workload compaction --steps 5 --warmup 1 > $O/bench_compaction.json 2> $O/bench_compaction.err || { echo "bench compaction failed"; tail $O/bench_compaction.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_compaction.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['round_build_ms'], d['last_round_stages_ms'], d['verified'])"
cp splinterdb_amd/librf_amd.so /tmp/librf_amd_k4.so && timeout -k 10 600 python3 tools/ab_chain.py /tmp/librf_amd_k4.so:RF_AMD_K4M=0 splinterdb_amd/librf_amd.so > $O/ab_chain.json 2> $O/ab_chain.err || { echo "ab failed"; tail $O/ab_chain.err; exit 1; }
cat $O/ab_chain.json
timeout -k 10 180 python3 tools/exit_bisect.py 9 > $O/m9.txt 2>&1; echo "mode 9 rc $?: $(tail -2 $O/m9.txt | tr '\n' ' ')"
