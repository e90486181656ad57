#!/bin/bash
# scratch iteration script for one gpurun call (overwritten per experiment)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
O=gpurun_out
PT_CHAIN=8 timeout -k 10 200 python tools/phase_times.py 1 64 1048575 > $O/pt1_chain8.txt 2>&1 || { tail -20 $O/pt1_chain8.txt; exit 1; }
tail -13 $O/pt1_chain8.txt
