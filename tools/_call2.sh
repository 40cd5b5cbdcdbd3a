export TMPDIR=/tmp
for v in 16_4 16_2 8_8 16_1; do echo "== $v"; timeout -k 10 60 ./tools/valu_probe_$v 10 || exit 1; done > gpurun_out/c2_probe.log 2>&1
cat gpurun_out/c2_probe.log
