# kernel trace of the compaction-chain bench (outputs under gpurun_out/prof_compaction/)
export TMPDIR=/tmp
O=gpurun_out/prof_compaction
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o comp -- python3 bench.py --workload compaction --steps 2 --warmup 0 --no-cpu-baseline > $O/kt.log 2>&1
