#!/bin/bash
# Round-3 shim checks on the GPU box: the whole -m gpu suite (shim tests first), then the
# engine's lookup round trip in each probe mode, then the shim's per-call costs.
cd "${GRAFT_REPO_ROOT:-.}" && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_shim.py \
  > gpurun_out/r03_shim_tests.log 2>&1 &&
for mw in mapped:flag copy:flag mapped:sync copy:sync; do
  echo -n "${mw} " >> gpurun_out/r03_probe_latency.txt &&
  RF_AMD_PROBE_MODE=${mw%%:*} RF_AMD_PROBE_WAIT=${mw##*:} timeout -k 10 120 python tools/probe_latency.py \
    >> gpurun_out/r03_probe_latency.txt || exit 1
done &&
timeout -k 10 600 python -u tools/shim_latency.py > gpurun_out/r03_shim_latency.json 2> gpurun_out/r03_shim_latency.err &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_gpu_filter_test.py \
  > gpurun_out/r03_filter_test.log 2>&1
