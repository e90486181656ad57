#!/bin/bash
# r05 call 10: K4m mismatch diagnosis (fuzz case 24), other new GPU tests (K4m off), C2 bench with the floor
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05d10
mkdir -p $O
RF_AMD_K4M=1 timeout -k 10 120 python tools/k4m_debug.py > $O/dbg1.txt 2>&1; echo "dbg1 rc $?"; cat $O/dbg1.txt
RF_AMD_K4M=0 timeout -k 10 120 python tools/k4m_debug.py > $O/dbg0.txt 2>&1 || { echo "dbg0 failed"; cat $O/dbg0.txt; exit 1; }
cat $O/dbg0.txt
RF_AMD_K4M=0 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rccl.py tests/test_gpu_server.py tests/test_gpu_trunk.py tests/test_gpu_probe_fast.py > $O/t2.log 2>&1 || { echo "tests2 failed"; tail -60 $O/t2.log; exit 1; }
tail -2 $O/t2.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $O/c2.json 2> $O/c2.err || { tail $O/c2.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c2.json').read()); print(d['value'], d['kernels']['probe']['ms'], d['roofline'], d['probe_floor'])"
