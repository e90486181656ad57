# A/B of librf_amd builds (tools/ab/librf_amd_<tag>.so) on the compaction chains, then C2/C3
# usage (on the box): bash tools/gpu_ab_comp.sh tagA tagB ...
mkdir -p gpurun_out
for r in 1 2; do for t in "$@"; do
  RF_AMD_LIB=tools/ab/librf_amd_$t.so timeout -k 10 300 python bench.py --workload compaction --no-cpu-baseline --steps 3 > gpurun_out/abc_$t.json 2> gpurun_out/abc_$t.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/abc_$t.json'));print('$t', d['value'], d['ms_per_step'], d['verified'], d.get('last_round_stages_ms',{}).get('cb_sort'))"
done; done
libs=""; for l in "$@"; do libs="$libs tools/ab/librf_amd_$l.so"; done
timeout -k 10 300 python tools/ab_probe2.py $libs > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
cat gpurun_out/ab.json
