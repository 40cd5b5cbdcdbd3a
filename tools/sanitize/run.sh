#!/bin/bash
# CPU build of the host planners under ASan + UBSan, then run it here (no
# GPU: every entry it calls is host-only). usage: bash tools/sanitize/run.sh [outdir]
# The library's sources are compiled with the sanitizers on the host side only
# (-fno-gpu-sanitize: the device code is compiled as usual and never launched).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=${1:-/tmp/gaplac_sanitize}
mkdir -p "$OUT"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fno-omit-frame-pointer \
  -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-gpu-sanitize \
  -o "$OUT/plan_sanitize" \
  "$ROOT/tools/sanitize/plan_sanitize.cpp" \
  "$ROOT/gaplac_amd/csrc/gaplac_kernels.hip" "$ROOT/gaplac_amd/csrc/gaplac_api.hip" "$ROOT/gaplac_amd/csrc/gaplac_dist.hip"
# leaks: the HIP runtime's own allocations at exit are not the planners'
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=0 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  "$OUT/plan_sanitize"
