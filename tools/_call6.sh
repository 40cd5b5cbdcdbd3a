export TMPDIR=/tmp
timeout -k 10 300 python bench.py --mode posterior --steps 5 --warmup 1 > gpurun_out/c6_post.json 2> gpurun_out/c6_post.err || { tail gpurun_out/c6_post.err; exit 1; }
timeout -k 10 300 python bench.py --mode rand --steps 5 --warmup 1 > gpurun_out/c6_rand.json 2> gpurun_out/c6_rand.err || { tail gpurun_out/c6_rand.err; exit 2; }
timeout -k 10 300 python bench.py --mode dist --steps 2 --warmup 1 > gpurun_out/c6_dist.json 2> gpurun_out/c6_dist.err || { tail gpurun_out/c6_dist.err; exit 3; }
timeout -k 10 300 python bench.py --mode select --steps 3 --warmup 1 > gpurun_out/c6_select.json 2> gpurun_out/c6_select.err || { tail gpurun_out/c6_select.err; exit 4; }
for f in post rand dist select; do grep -h '^{' gpurun_out/c6_$f.json | cut -c1-700; done
