export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/c1_pytest.log 2>&1 || { tail -30 gpurun_out/c1_pytest.log; exit 1; }
tail -2 gpurun_out/c1_pytest.log
timeout -k 10 120 ./tools/mfma_f64_rate > gpurun_out/c1_mfma.log 2>&1 || exit 2
cat gpurun_out/c1_mfma.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --skip-cpu > gpurun_out/c1_bench.json 2> gpurun_out/c1_bench.err || exit 3
cut -c 1-400 gpurun_out/c1_bench.json
