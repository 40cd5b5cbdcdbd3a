# snake default: distributed / configs / bench-leg GPU tests
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_dist_replay.py tests/test_gpu_configs.py tests/test_gpu_bench_dist.py tests/test_gpu_nccl.py > gpurun_out/r06sd_tests.log 2>&1
