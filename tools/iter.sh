#!/bin/bash
# r05 call 41: K6 ablations + phase stamps on the reworked K6; final round-5 lines and kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05d41
mkdir -p $O
AB_NOPROBE=1 timeout -k 10 300 python3 tools/ab_build.py tools/ab/librf_amd_{base,s1,s2,s3}.so > $O/ab.json 2> $O/ab.err || { echo "ab failed"; tail $O/ab.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab.json')); [print(k, v['assemble'], v['cb_sort'], v['build_total']) for k,v in d['stage_ms_median'].items()]"
timeout -k 10 180 python3 tools/phase_times.py 3 > $O/phase_k3.txt 2>&1 || { echo "phase failed"; tail $O/phase_k3.txt; exit 1; }
cat $O/phase_k3.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o c2 -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $O/kt.log 2>&1 || { echo "kernel trace failed"; exit 1; }
timeout -k 10 400 python3 bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench c2 failed"; tail $O/bench_c2.err; exit 1; }
for w in c3 c4; do
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline --pmc none > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; exit 1; }
done
timeout -k 10 300 python3 bench.py --workload c5 --pmc none > $O/bench_c5.json 2> $O/bench_c5.err || { echo "bench c5 failed"; exit 1; }
timeout -k 10 300 python3 bench.py --workload compaction --steps 5 --warmup 1 > $O/bench_compaction.json 2> $O/bench_compaction.err || { echo "bench compaction failed"; exit 1; }
for w in c2 c3 c4 c5 compaction; do
python3 -c "
import json; d=json.loads(open('$O/bench_$w.json').read().strip().splitlines()[-1]); k=d.get('kernels',{}); print('$w', d['value'], d['ms_per_step'], {a: (b['ms'] if isinstance(b, dict) else b) for a,b in k.items()}, d.get('last_round_stages_ms'), d['roofline']['frac'], d.get('probe_floor',{}).get('probe_over_floor'), d['verified'])" | cut -c1-700
done
