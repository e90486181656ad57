# incremental-build check on the box: K4 phase stamps at compaction round 8, the incremental
# GPU tests, and the compaction bench line (outputs under gpurun_out/)
mkdir -p gpurun_out
PT_CHAIN=8 timeout -k 10 150 python tools/phase_times.py 1 64 1048575 > gpurun_out/phases_chain_k1.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_compaction.py tests/test_gpu_fuzz.py tests/test_gpu_shim.py tests/test_gpu_poison.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_merge.log 2>&1 || { tail -30 gpurun_out/t_merge.log; exit 1; }
tail -1 gpurun_out/t_merge.log
timeout -k 10 300 python bench.py --workload compaction --no-cpu-baseline > gpurun_out/b_comp.json 2> gpurun_out/b_comp.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/b_comp.json'));print(d['value'], d['verified'], d.get('last_round_stages_ms'), d['ms_per_step'])"
grep -v amdgpu.ids gpurun_out/phases_chain_k1.txt
