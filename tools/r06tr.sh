# tail gather at configs[3]: one-GPU replay of rank 0 (the gather's root) and rank 7 over tail lengths
export PYTHONUNBUFFERED=1
O=gpurun_out/r06tr_replay_tail.jsonl
timeout -k 10 500 python -u tools/dist_replay.py --N 65536 --ranks 8 --local 0 --bw 200 --depth 2 --chunk 2 --big 1 --alone 1 \
  --iters 4 --tail 0 48 64 80 96 112 128 --gbw 50 --out $O > gpurun_out/r06tr_a.log 2>&1 && \
timeout -k 10 300 python -u tools/dist_replay.py --N 65536 --ranks 8 --local 0 7 --bw 200 --depth 2 --chunk 2 --big 1 --alone 1 \
  --iters 4 --tail 80 --gbw 25 100 --out $O > gpurun_out/r06tr_b.log 2>&1 && \
timeout -k 10 300 python -u tools/dist_replay.py --N 65536 --ranks 8 --local 7 --bw 200 --depth 2 --chunk 2 --big 1 --alone 1 \
  --iters 4 --tail 0 --out $O > gpurun_out/r06tr_c.log 2>&1
