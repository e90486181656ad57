#!/bin/bash
# scratch iteration script for one gpurun call (overwritten per experiment)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/gt_full.log 2>&1 || { tail -40 $O/gt_full.log; exit 1; }
tail -1 $O/gt_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/profile_round.sh r04b
