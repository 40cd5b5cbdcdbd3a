# configs[3] job replay: which held ops (alone 1 / 2 / 3) balance the ranks, with and without the tail gather
export PYTHONUNBUFFERED=1
O=gpurun_out/r06ta_replay_job.jsonl
for al in 2 3; do
timeout -k 10 400 python -u tools/dist_replay.py --N 65536 --ranks 8 --job --bw 200 --depth 2 --chunk 2 --big 1 --alone $al \
  --iters 4 --tail 0 48 --gbw 50 --out $O > gpurun_out/r06ta_$al.log 2>&1 || exit 1
done
