#!/bin/bash
# r05 call 28: final validation: full GPU suite, smoke, the driver's default bench command
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05d28
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/ > $O/t.log 2>&1 || { echo "tests failed"; grep -v "^  File" $O/t.log | tail -40; exit 1; }
tail -2 $O/t.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['build_mkeys_s'], d['probe_mkeys_s'], d['roofline'], d['probe_floor']['probe_over_floor'], d['verified'], d['cpu_baseline']['value'])"
