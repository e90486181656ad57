# round-end check on the box: GPU tests, smoke(), the default bench line, the compaction
# line and its kernel trace (outputs under gpurun_out/)
mkdir -p gpurun_out
bash tools/gpu_tests.sh || { tail -30 gpurun_out/gputest.log; exit 1; }
tail -1 gpurun_out/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_default.json'));print('c2', d['value'], d['ms_per_step'], d['verified'], d['roofline']['frac'])"
timeout -k 10 300 python bench.py --workload compaction > gpurun_out/bench_compaction.json 2> gpurun_out/bench_compaction.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_compaction.json'));print('compaction', d['value'], d['ms_per_step'], d['verified'], d['dropin_latency'])"
bash tools/prof_compaction.sh || exit 1
