export TMPDIR=/tmp; R=r04e; mkdir -p gpurun_out/$R
timeout -k 10 60 ./tools/bin/diag_probe > gpurun_out/$R/diag_probe.txt 2>&1; rc=$?
grep -v "^  v1" gpurun_out/$R/diag_probe.txt | head -60
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_schedules.py tests/test_gpu_configs.py tests/test_gpu_robust.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest.log 2>&1 || { tail -30 gpurun_out/$R/pytest.log; exit 2; }
tail -1 gpurun_out/$R/pytest.log
timeout -k 10 300 python -u tools/ab.py $R --reps 2 --ns 16384,4096 --select cur v2:lib=tools/bin/lib_v2.so || exit 3
bash tools/gpu_trace.sh $R 4096 > gpurun_out/$R/t4096.txt 2>&1 || exit 5
cat gpurun_out/$R/t4096.txt
