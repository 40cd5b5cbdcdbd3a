# configs[3] whole-job replay (snake layout): the schedule options re-checked as a job (every rank)
export PYTHONUNBUFFERED=1
O=gpurun_out/r06jo_replay_job_options.jsonl
run() { timeout -k 10 300 python -u tools/dist_replay.py --N 65536 --ranks 8 --job --bw 200 --iters 4 --tail 0 --snake 1 --out $O "$@" >> gpurun_out/r06jo.log 2>&1; }
run --depth 3 --chunk 2 --big 1 --alone 1 && \
run --depth 4 --chunk 2 --big 1 --alone 1 && \
run --depth 2 --chunk 1 --big 1 --alone 1 && \
run --depth 2 --chunk 4 --big 1 --alone 1 && \
run --depth 2 --chunk 2 --big 1 --alone 0 && \
run --depth 2 --chunk 2 --big 0 --alone 1
