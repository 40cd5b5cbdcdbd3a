export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_posterior.py -x -v --timeout 120 --timeout-method thread > gpurun_out/c5_post.log 2>&1; rc=$?
tail -30 gpurun_out/c5_post.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/c5_all.log 2>&1 || { tail -30 gpurun_out/c5_all.log; exit 2; }
tail -3 gpurun_out/c5_all.log
