#!/bin/bash
# The bulk tile kernel alone (tools/bulk_probe.hip) over matrix orders, trailing sizes and
# depths, for every built variant (tools/bin/bulk_probe*), then one PMC pass (clock and
# MFMA busy) at the 16k and 64k shapes.   usage: bash tools/bulk_probe_sweep.sh OUTDIR [pmc]
set -e
O=${1:-gpurun_out/bulk_probe}
mkdir -p $O
export TMPDIR=/tmp
for args in "129 120 1024" "129 80 1024" "129 120 512" "513 500 1024"; do
  for P in tools/bin/bulk_probe tools/bin/bulk_probe_*; do
    [ -x $P ] || continue
    echo "variant $P"; timeout -k 5 60 $P $args 5
  done
done
[ "$2" = pmc ] || exit 0
for args in "129 120 1024" "513 500 1024"; do
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/pmc_${args// /_} -o run --output-format csv -- tools/bin/bulk_probe $args 3
done
