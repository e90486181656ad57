#!/bin/bash
# quick A/B: GPU tests, then C2 x2, C3, C5 bench lines (kernel ms) -- one gpurun call
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gt.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gt.log; [ $rc -eq 0 ] || exit $rc
for w in ${@:-c2 c2 c3 c5}; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-e2e > gpurun_out/b_$w.json 2> gpurun_out/b_$w.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/b_$w.json'));print('$w',d['value'],d['ms_per_step'],d['verified'],{k:v['ms'] for k,v in d['kernels'].items()})"
done
