export TMPDIR=/tmp; R=r04g; mkdir -p gpurun_out/$R
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_nccl.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$R/pytest.log 2>&1 || { tail -40 gpurun_out/$R/pytest.log; exit 1; }
tail -3 gpurun_out/$R/pytest.log
bash tools/dist_bench.sh $R || exit 2
