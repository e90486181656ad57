#!/bin/bash
# r05 call 17: K4m v2.4 (new-entry loads and old-run DMA on different waves) + 32-bit SWAR decode in the probe fast path
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05d17
mkdir -p $O
RF_AMD_K4M=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_compaction.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_probe_fast.py tests/test_gpu_boundary.py > $O/t.log 2>&1 || { echo "tests failed"; grep -v "^  File" $O/t.log | tail -50; exit 1; }
tail -2 $O/t.log
cp splinterdb_amd/librf_amd.so /tmp/librf_amd_k4m.so && timeout -k 10 600 python3 tools/ab_chain.py splinterdb_amd/librf_amd.so /tmp/librf_amd_k4m.so:RF_AMD_K4M=1 > $O/ab_chain.json 2> $O/ab_chain.err || { echo "ab failed"; tail $O/ab_chain.err; exit 1; }
cat $O/ab_chain.json
RF_AMD_K4M=1 PT_CHAIN=8 timeout -k 10 300 python tools/phase_times.py 5 64 1048575 > $O/pt5_chain8.txt 2>&1 || { tail -20 $O/pt5_chain8.txt; exit 1; }
tail -14 $O/pt5_chain8.txt
timeout -k 10 600 python3 tools/ab_probe2.py tools/ab/librf_amd_head.so splinterdb_amd/librf_amd.so tools/ab/librf_amd_head.so splinterdb_amd/librf_amd.so > $O/ab_probe.json 2> $O/ab_probe.err || { echo "ab probe failed"; tail $O/ab_probe.err; exit 1; }
cat $O/ab_probe.json
