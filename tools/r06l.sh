export TMPDIR=/tmp; mkdir -p gpurun_out/r06l
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_switches.py tests/test_gpu_schedules.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06l/pytest.log 2>&1; tail -3 gpurun_out/r06l/pytest.log
grep -q " passed" gpurun_out/r06l/pytest.log && ! grep -q "failed\|error" gpurun_out/r06l/pytest.log || exit 1
timeout -k 10 600 python tools/ab.py r06l --reps 2 --ns 16384,8192,4096 --select cur nopair:lib=tools/bin/lib_nopair.so
