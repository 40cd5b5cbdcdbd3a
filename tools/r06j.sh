export TMPDIR=/tmp; mkdir -p gpurun_out/r06j
timeout -k 5 120 tools/bin/bulk_probe_clk 129 113 1024 20 1 > gpurun_out/r06j/probe.txt 2>&1 || exit 1
grep clock gpurun_out/r06j/probe.txt
for arm in clk clk_skip2; do
GAPLAC_LIB_PATH=tools/bin/lib_$arm.so timeout -k 10 200 python tools/clk_eval.py > gpurun_out/r06j/$arm.txt 2>&1 || exit 2
echo "== $arm"; grep "clk slot" gpurun_out/r06j/$arm.txt | tail -13
done
