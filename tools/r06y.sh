export TMPDIR=/tmp; mkdir -p gpurun_out/r06y
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_switches.py tests/test_gpu_schedules.py tests/test_gpu_robust.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06y/pytest.log 2>&1; tail -3 gpurun_out/r06y/pytest.log
grep -q " passed" gpurun_out/r06y/pytest.log && ! grep -q "failed\|error" gpurun_out/r06y/pytest.log || exit 1
timeout -k 10 900 python tools/ab.py r06y --reps 3 --ns 16384,12000 cur nopre:lib=tools/bin/lib_noprefix.so
