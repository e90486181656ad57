# compaction-chain tests + bench line (logs under gpurun_out/)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_compaction.py -x -v --timeout 500 --timeout-method thread > gpurun_out/gputest_compaction.log 2>&1 && \
timeout -k 10 400 python bench.py --workload compaction --steps 5 --warmup 1 > gpurun_out/bench_compaction.json 2> gpurun_out/bench_compaction.err
