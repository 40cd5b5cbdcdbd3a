export TMPDIR=/tmp; R=r04d; mkdir -p gpurun_out/$R
timeout -k 10 300 python -u -m pytest tests/test_gpu_schedules.py tests/test_gpu_robust.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest.log 2>&1 || { tail -30 gpurun_out/$R/pytest.log; exit 1; }
tail -1 gpurun_out/$R/pytest.log
timeout -k 10 900 python -u tools/ab.py $R --reps 2 --ns 16384,4096 --select cur nodeq:lib=tools/bin/lib_nodeq.so gw8:GAPLAC_SINGLE_GW=8 || exit 2
