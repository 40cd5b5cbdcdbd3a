# snake layout: the distributed GPU tests, then the whole-job replay at configs[3] with / without the snake and the tail gather
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_dist_replay.py > gpurun_out/r06sn_tests.log 2>&1 && \
timeout -k 10 900 python -u tools/dist_replay.py --N 65536 --ranks 8 --job --bw 200 --depth 2 --chunk 2 --big 1 --alone 1 \
  --iters 4 --tail 0 48 64 --snake 1 --gbw 50 --out gpurun_out/r06sn_replay_job.jsonl > gpurun_out/r06sn.log 2>&1
