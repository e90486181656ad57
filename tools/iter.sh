#!/bin/bash
# r06 call 10: K4m2 diagnostics -- coarse buckets handed back per round
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
cp splinterdb_amd/librf_amd.so /tmp/k4m1.so
RF_AMD_DIAG_OVERFLOW=1 AB_R=8 AB_REPS=1 timeout -k 10 300 python3 tools/ab_chain.py /tmp/k4m1.so:RF_AMD_K4M=1 splinterdb_amd/librf_amd.so > $O/ab_r8.json 2> $O/ab_r8.err || { echo "ab failed"; tail -5 $O/ab_r8.err; exit 1; }
cat $O/ab_r8.json; grep "handed back" $O/ab_r8.err
