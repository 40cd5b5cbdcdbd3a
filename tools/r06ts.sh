# tail gather: the standalone tail at T = 77 / 80 (sim order on / off), and the replayed job's other ranks over tail lengths
export PYTHONUNBUFFERED=1
O=gpurun_out/r06ts_replay_tail.jsonl
timeout -k 10 300 python tools/ab.py r06ts --reps 3 --ns 9855,10239 cur nosim:GAPLAC_TAIL_SIM=0 > gpurun_out/r06ts_ab.log 2>&1 && \
timeout -k 10 600 python -u tools/dist_replay.py --N 65536 --ranks 8 --local 3 7 --bw 200 --depth 2 --chunk 2 --big 1 --alone 1 \
  --iters 4 --tail 64 80 96 --gbw 50 --out $O > gpurun_out/r06ts_a.log 2>&1 && \
GAPLAC_TAIL_SIM=0 timeout -k 10 300 python -u tools/dist_replay.py --N 65536 --ranks 8 --local 0 --bw 200 --depth 2 --chunk 2 --big 1 --alone 1 \
  --iters 4 --tail 80 96 --gbw 50 --out $O > gpurun_out/r06ts_b.log 2>&1
