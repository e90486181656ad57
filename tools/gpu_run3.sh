# bench: default (C2) line with the reference CPU baseline, then C3, C4, C5 lines
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err && \
timeout -k 10 300 python bench.py --workload c3 --steps 10 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err && \
timeout -k 10 300 python bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err && \
timeout -k 10 400 python bench.py --workload c5 --steps 10 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
