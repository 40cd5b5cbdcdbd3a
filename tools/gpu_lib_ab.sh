#!/bin/bash
# Library A/B: arms as tools/ab.py takes them; headline + configs[1] + 64k sizes, gradient.
# usage: bash tools/gpu_lib_ab.sh TAG ARM...
T=$1; shift
timeout -k 10 1000 python tools/ab.py $T --reps 3 --ns 16384,4096,65536 --grad "$@"
