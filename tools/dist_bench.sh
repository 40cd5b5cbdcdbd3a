export TMPDIR=/tmp; mkdir -p gpurun_out
set -o pipefail
timeout -k 10 150 python bench.py --mode single --steps 3 --warmup 1 > gpurun_out/d_single.json 2>&1 && tail -1 gpurun_out/d_single.json | cut -c1-400 &&
timeout -k 10 150 python bench.py --mode dist --steps 3 --warmup 1 > gpurun_out/d_dist1.json 2>&1 && tail -1 gpurun_out/d_dist1.json | cut -c1-400 &&
timeout -k 10 200 python bench.py --mode dist --loopback 2 --steps 3 --warmup 1 > gpurun_out/d_loop2.json 2>&1 && tail -1 gpurun_out/d_loop2.json | cut -c1-400 &&
timeout -k 10 200 python bench.py --mode dist --loopback 8 --steps 3 --warmup 1 > gpurun_out/d_loop8.json 2>&1 && tail -1 gpurun_out/d_loop8.json | cut -c1-400
