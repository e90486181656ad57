#!/bin/bash
# r06 session 2, call 6: server pass diagnostics (requests per pass, cuts) and outstanding states at reaps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06s2f
mkdir -p $O
cp splinterdb_amd/librf_amd.so $O/librf_amd_default.so.bak
AD_REPS=9 AD_ONLY=shim timeout -k 10 200 python3 -u tools/async_driven.py > $O/ad_1.json 2> $O/ad_1.err || { echo ad failed; tail -20 $O/ad_1.err; exit 1; }
echo "default: $(cat $O/ad_1.json)"
cp tools/ab/librf_amd_srvprof.so splinterdb_amd/librf_amd.so
RF_AMD_SUBMIT_PROFILE=1 RF_SHIM_SUBMIT_PROFILE=1 AD_REPS=9 AD_ONLY=shim timeout -k 10 200 python3 -u tools/async_driven.py > $O/ad_prof.json 2> $O/ad_prof.err || { echo ad failed; tail -20 $O/ad_prof.err; exit 1; }
echo "prof: $(cat $O/ad_prof.json)"; grep "profile\|passes\|reaps" $O/ad_prof.err
cp $O/librf_amd_default.so.bak splinterdb_amd/librf_amd.so
timeout -k 10 300 python3 tools/trunk_latency.py > $O/trunk_latency.json 2> $O/trunk_latency.err || { echo trunk latency failed; tail -5 $O/trunk_latency.err; exit 1; }
cat $O/trunk_latency.json
