export TMPDIR=/tmp; mkdir -p gpurun_out/r06i
timeout -k 5 120 tools/bin/bulk_probe_clk 129 113 1024 20 1 > gpurun_out/r06i/probe.txt 2>&1 || exit 1
cat gpurun_out/r06i/probe.txt
GAPLAC_LIB_PATH=tools/bin/lib_clk.so timeout -k 10 200 python bench.py --steps 5 --warmup 2 --skip-cpu --no-extra --profile-steps 3 > gpurun_out/r06i/bench.json 2> gpurun_out/r06i/clk.txt || exit 2
grep "clk slot" gpurun_out/r06i/clk.txt | tail -30
