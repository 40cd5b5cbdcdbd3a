export TMPDIR=/tmp; R=r04j; mkdir -p gpurun_out/$R
timeout -k 10 200 python -u -m pytest tests/test_gpu_robust.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$R/pytest.log 2>&1 || { tail -30 gpurun_out/$R/pytest.log; exit 1; }
tail -1 gpurun_out/$R/pytest.log
timeout -k 10 600 python -u tools/ab.py $R --reps 2 --ns 4096,16384 cur r03:lib=tools/bin/lib_r03.so || exit 3
