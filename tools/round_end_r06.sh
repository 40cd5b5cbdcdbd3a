#!/bin/bash
# Round-6 end pass on one box: every GPU test, smoke, the round profile (kernel-trace stats,
# PMC traffic passes, full bench line: tools/profile_round.sh), the evaluation timeline, and
# the gradient / posterior / rand bench lines.   usage: bash tools/round_end_r06.sh rNN
R=${1:-r06end}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$R/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$R/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$R/smoke.log 2>&1 || { tail -20 gpurun_out/$R/smoke.log; exit 2; }
cat gpurun_out/$R/smoke.log
bash tools/profile_round.sh $R || exit 3
python tools/timeline2.py gpurun_out/$R/trace > gpurun_out/$R/timeline.txt || exit 4
python tools/launch_list.py gpurun_out/$R/trace > gpurun_out/$R/launches.txt || exit 4
head -20 gpurun_out/$R/timeline.txt
for m in grad posterior rand; do
  timeout -k 10 300 python bench.py --mode $m --steps 5 --warmup 1 > gpurun_out/$R/bench_$m.json 2> gpurun_out/$R/bench_$m.err || exit 5
  cut -c1-240 gpurun_out/$R/bench_$m.json
done
