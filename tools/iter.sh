#!/bin/bash
# r05 call 11: full GPU suite (K4m on, opt-in direct placement), K4m A/B vs HEAD~, phase stamps, C2 bench with the floor
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05d11
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/ > $O/t.log 2>&1 || { echo "tests failed"; grep -v "^  File" $O/t.log | tail -40; exit 1; }
tail -2 $O/t.log
timeout -k 10 600 python3 tools/ab_chain.py tools/ab/librf_amd_head.so splinterdb_amd/librf_amd.so > $O/ab_chain.json 2> $O/ab_chain.err || { echo "ab failed"; tail $O/ab_chain.err; exit 1; }
cat $O/ab_chain.json
PT_CHAIN=8 timeout -k 10 300 python tools/phase_times.py 5 64 1048575 > $O/pt5_chain8.txt 2>&1 || { tail -20 $O/pt5_chain8.txt; exit 1; }
tail -14 $O/pt5_chain8.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $O/c2.json 2> $O/c2.err || { tail $O/c2.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c2.json').read()); print(d['value'], d['kernels']['probe']['ms'], d['roofline'], d['probe_floor'])"
