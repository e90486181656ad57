#!/bin/bash
# Round-3 iteration on the GPU box: the -m gpu suite (without the long filter_test.c run), the
# shim's per-call costs, the incremental K4 A/B (merge path vs direct placement), the compaction bench, and per-phase stamps of K4 and K6 at round 8 of
# the compaction chains (diagnostics library).
cd "${GRAFT_REPO_ROOT:-.}" && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  --deselect tests/test_gpu_filter_test.py > gpurun_out/r03_gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/k4_ab.py 64 5 > gpurun_out/r03_k4_ab.json 2> gpurun_out/r03_k4_ab.err &&
timeout -k 10 300 python bench.py --workload compaction --steps 3 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r03_bench_compaction.json 2> gpurun_out/r03_bench_compaction.err &&
timeout -k 10 600 python -u tools/shim_latency.py > gpurun_out/r03_shim_latency.json 2> gpurun_out/r03_shim_latency.err &&
PT_CHAIN=8 timeout -k 10 300 python tools/phase_times.py 1 64 1048575 > gpurun_out/r03_phases_chain_k4.txt 2>&1 &&
PT_CHAIN=8 timeout -k 10 300 python tools/phase_times.py 3 64 1048575 > gpurun_out/r03_phases_chain_k6.txt 2>&1
