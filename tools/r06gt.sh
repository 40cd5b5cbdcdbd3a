# gradient / posterior: the tail length in the extra-rows modes (the main matrix's last columns as per-column launches there)
export PYTHONUNBUFFERED=1
timeout -k 10 900 python tools/ab.py r06gt --reps 2 --ns "" --grad --posterior cur t48:GAPLAC_TAIL_S=48 t24:GAPLAC_TAIL_S=24 t8:GAPLAC_TAIL_S=8 > gpurun_out/r06gt.log 2>&1
