mkdir -p gpurun_out
(nproc; python -c "import os;print('affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max; cat /proc/meminfo | head -3; lscpu | head -25) > gpurun_out/host.txt 2>&1
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > gpurun_out/gputest.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
