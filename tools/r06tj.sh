# tail gather at configs[3]: every rank replayed, the job's prediction per tail length
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u tools/dist_replay.py --N 65536 --ranks 8 --job --bw 200 --depth 2 --chunk 2 --big 1 --alone 1 \
  --iters 4 --tail 0 32 48 64 80 --gbw 50 --out gpurun_out/r06tj_replay_job.jsonl > gpurun_out/r06tj.log 2>&1
