#!/bin/bash
# r05 call 37: GPU test suite with the block-aligned K6 runs; K6 A/B; compaction chain
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05d37
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1 || { echo "gpu tests failed"; tail -30 $O/gputest.txt; exit 1; }
tail -2 $O/gputest.txt
timeout -k 10 300 python3 tools/ab_build.py tools/ab/librf_amd_k6{a,g,h,i}.so > $O/ab.json 2> $O/ab.err || { echo "ab failed"; tail $O/ab.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab.json')); print(d['images_identical'], d['probes_identical'], d['all_found']); [print(k, v['assemble'], v['build_total']) for k,v in d['stage_ms_median'].items()]"
timeout -k 10 300 python3 bench.py --workload compaction --steps 5 --warmup 1 > $O/bench_compaction.json 2> $O/bench_compaction.err || { echo "bench compaction failed"; tail $O/bench_compaction.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_compaction.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], json.dumps(d.get('last_round_stages', d.get('stages', {})))[:600])"
