#!/bin/bash
# r06 call 29: completion threads pinned to the caller's LLC (RF_SHIM_PIN_THREADS 0 vs 1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06zc
mkdir -p $O
for i in 1 2; do
for P in 0 1; do
  RF_SHIM_PIN_THREADS=$P AD_REPS=9 timeout -k 10 300 python3 -u tools/async_driven.py > $O/ad_p${P}_$i.json 2> $O/ad_p${P}_$i.err || { echo ad failed; tail -40 $O/ad_p${P}_$i.err; exit 1; }
  echo "pin=$P"; cat $O/ad_p${P}_$i.json
done
done
cat /sys/devices/system/cpu/cpu0/cache/index3/shared_cpu_list; taskset -p $$
