set -e
bash tools/bulk_probe_sweep.sh gpurun_out/r04x > gpurun_out/r04x_bulk_probe.txt 2>&1
grep -v "^W20\|^E20" gpurun_out/r04x_bulk_probe.txt | tail -30
timeout -k 10 900 python tools/ab.py r04x --reps 3 --ns 16384 --grad --tests tests/test_gpu_parity.py,tests/test_gpu_grad.py,tests/test_gpu_schedules.py,tests/test_gpu_posterior.py cur dma:lib=tools/bin/lib_dma.so
