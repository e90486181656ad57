mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_shim.py tests/test_shim_boundary.py -x -v --timeout 600 --timeout-method thread > gpurun_out/gputest_shim.log 2>&1
