#!/bin/bash
# r05 call 43: K4m merge read-ahead A/B on the round-8 chain
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05d43
mkdir -p $O
AB_REPS=5 timeout -k 10 500 python3 tools/ab_chain.py tools/ab/librf_amd_base.so tools/ab/librf_amd_k4r.so > $O/chain.json 2> $O/chain.err || { echo "chain failed"; tail $O/chain.err; exit 1; }
cat $O/chain.json | cut -c1-1500
