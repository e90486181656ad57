# A/B run: probe-affecting GPU tests, then tools/ab_probe2.py over tools/ab/*.so
# usage (on the box): bash tools/gpu_ab.sh libA libB ...   (names under tools/ab/)
mkdir -p gpurun_out
if [ -z "$AB_SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "not two_ranks" > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
fi
libs=""; for l in "$@"; do libs="$libs tools/ab/librf_amd_$l.so"; done
timeout -k 10 300 python tools/ab_probe2.py $libs > gpurun_out/ab.json 2> gpurun_out/ab.err; rc=$?
cat gpurun_out/ab.json; exit $rc
