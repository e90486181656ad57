#!/bin/bash
# r06 session 3, call 3: floor with gathers independent of the key loads (KM=3), split rerun
# at C2's and C3's shapes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06s3c
mkdir -p $O
FB_SET=2 timeout -k 10 120 ./tools/floor_bench $((64<<20)) 8 8388608 "C2 shape" > $O/split.txt 2>&1 || { echo c2 failed; cat $O/split.txt; exit 1; }
FB_SET=2 timeout -k 10 180 ./tools/floor_bench $((256<<20)) 256 2097152 "C3 shape" >> $O/split.txt 2>&1 || { echo c3 failed; cat $O/split.txt; exit 1; }
cat $O/split.txt
