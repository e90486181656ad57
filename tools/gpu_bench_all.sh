mkdir -p gpurun_out
bash tools/gpu_tests.sh || { tail -30 gpurun_out/gputest.log; exit 1; }
tail -1 gpurun_out/gputest.log
for w in c2 c3 c4 c5; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-e2e > gpurun_out/b_$w.json 2> gpurun_out/b_$w.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/b_$w.json'));print('$w', d['value'], d['ms_per_step'], d['verified'], d['roofline']['frac'], d['kernels']['probe']['ms'])"
done
