#!/bin/bash
# r06 call 33: the idle poll hands its window to the next pass
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06zg
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_server.py tests/test_gpu_shim.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
AD_REPS=9 timeout -k 10 300 python3 -u tools/async_driven.py > $O/ad_$i.json 2> $O/ad_$i.err || { echo ad failed; tail -40 $O/ad_$i.err; exit 1; }
cat $O/ad_$i.json
done
cp tools/ab/librf_amd_srvprof.so splinterdb_amd/librf_amd.so
RF_AMD_SUBMIT_PROFILE=1 AD_ONLY=shim timeout -k 10 300 python3 -u tools/async_driven.py > $O/ad_prof.json 2> $O/ad_prof.err || { echo ad failed; tail -40 $O/ad_prof.err; exit 1; }
cat $O/ad_prof.json; grep "profile\|passes" $O/ad_prof.err
