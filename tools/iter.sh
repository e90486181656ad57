#!/bin/bash
# scratch iteration script for one gpurun call (overwritten per experiment)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 400 python3 tools/ab_probe2.py tools/ab/librf_amd_nt1024.so tools/ab/librf_amd_nt512.so tools/ab/librf_amd_nt256.so > $O/ab_nt.json 2> $O/ab_nt.err || { tail -20 $O/ab_nt.err; exit 1; }
cat $O/ab_nt.json
