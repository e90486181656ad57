#!/bin/bash
# r05 call 29: probe keys requested before the wave table / plan loads: parity, A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05d29
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_probe_fast.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_boundary.py tests/test_gpu_configs.py > $O/t.log 2>&1 || { echo "tests failed"; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 600 python3 tools/ab_probe2.py tools/ab/librf_amd_head.so splinterdb_amd/librf_amd.so tools/ab/librf_amd_head.so splinterdb_amd/librf_amd.so > $O/ab_probe.json 2> $O/ab_probe.err || { echo "ab probe failed"; tail $O/ab_probe.err; exit 1; }
cat $O/ab_probe.json
timeout -k 10 300 python3 bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --pmc none > $O/c3.json 2> $O/c3.err || { tail $O/c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c3.json').read().strip().splitlines()[-1]); print(d['value'], d['kernels']['probe']['ms'], d['probe_floor'])"
