#!/bin/bash
# scratch iteration script for one gpurun call (overwritten per experiment)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
O=gpurun_out
for mode in default nosdma; do
  if [ $mode = nosdma ]; then export HSA_ENABLE_SDMA=0; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_$mode.json 2> $O/b_$mode.err || { tail -20 $O/b_$mode.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_$mode.json'));print('$mode', d['value'], d['e2e_pcie_mkeys_s'], d['e2e_pcie_serial_mkeys_s'], d['e2e_pcie_hashes_mkeys_s'], d['verified'])"
done
