#!/bin/bash
# The bulk tile kernel alone (tools/bulk_probe.hip) over matrix orders, trailing sizes and
# depths, then one PMC pass (clock and MFMA busy) at the 16k and 64k shapes.
# usage: bash tools/bulk_probe_sweep.sh OUTDIR
set -e
O=${1:-gpurun_out/bulk_probe}
mkdir -p $O
export TMPDIR=/tmp
P=tools/bin/bulk_probe
for args in "129 120 1024" "129 80 1024" "129 120 512" "513 120 1024" "513 500 1024" "136 120 1024"; do
  for V in "" _dma; do
    [ -x $P$V ] || continue
    echo "variant ${V:-base}"; timeout -k 5 60 $P$V $args 5
  done
done
for args in "129 120 1024" "513 500 1024"; do
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/pmc_${args// /_} -o run --output-format csv -- $P $args 3
done
