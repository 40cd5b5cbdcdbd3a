# deeper deferral below 256 tile columns, with and without the split
timeout -k 10 1000 python tools/ab.py r06z --reps 3 --ns 16384,12000 cur d3s:lib=tools/bin/lib_d3s.so d4s:lib=tools/bin/lib_d4s.so d3n:lib=tools/bin/lib_d3n.so d4n:lib=tools/bin/lib_d4n.so
