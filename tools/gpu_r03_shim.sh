#!/bin/bash
# Round-3 checks on the GPU box: the whole -m gpu suite (the drop-in's filter_test.c run last),
# the engine's lookup round trip, the shim's per-call costs, the compaction bench line and the
# probe-kernel A/B (k_probe vs the pipelined k_probe_pipe).
cd "${GRAFT_REPO_ROOT:-.}" && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
  --deselect tests/test_gpu_filter_test.py > gpurun_out/r03_gpu_tests.log 2>&1 &&
timeout -k 10 300 python tools/probe_pipe_ab.py c2 0 7 8 4 > gpurun_out/r03_pipe_ab.txt 2>&1 &&
timeout -k 10 300 python tools/probe_pipe_ab.py c3 0 7 8 4 >> gpurun_out/r03_pipe_ab.txt 2>&1 &&
echo -n "default " > gpurun_out/r03_probe_latency.txt &&
timeout -k 10 120 python tools/probe_latency.py >> gpurun_out/r03_probe_latency.txt &&
echo -n "no-small-path " >> gpurun_out/r03_probe_latency.txt &&
RF_AMD_PROBE_SMALL=0 timeout -k 10 120 python tools/probe_latency.py >> gpurun_out/r03_probe_latency.txt &&
timeout -k 10 600 python -u tools/shim_latency.py > gpurun_out/r03_shim_latency.json 2> gpurun_out/r03_shim_latency.err &&
timeout -k 10 300 python bench.py --workload compaction --steps 3 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r03_bench_compaction.json 2> gpurun_out/r03_bench_compaction.err &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_gpu_filter_test.py \
  > gpurun_out/r03_filter_test.log 2>&1
