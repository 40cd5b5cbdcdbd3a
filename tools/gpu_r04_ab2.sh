#!/bin/bash
# round-4 A/B bundle: tail size after the LDS-DMA change, large-launch bulk kernel at 64k
set -e
timeout -k 10 500 python tools/ab.py r04zd --reps 3 --ns 16384 t80:GAPLAC_TAIL_S=80 t64:GAPLAC_TAIL_S=64 t72:GAPLAC_TAIL_S=72 t88:GAPLAC_TAIL_S=88
timeout -k 10 500 python tools/ab.py r04ze --reps 3 --ns 65536 big:GAPLAC_BULK_BIG=1 nobig:GAPLAC_BULK_BIG=0
