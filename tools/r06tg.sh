# tail gather: the distributed GPU tests (loopback, gloo, tail, replay), then the configs / bench-leg tests
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_dist_replay.py > gpurun_out/r06tg_dist.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_bench_dist.py > gpurun_out/r06tg_more.log 2>&1
