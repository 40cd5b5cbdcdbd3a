#!/bin/bash
# Build the library as it was at a git commit (an A/B control arm, e.g. the previous round's
# final state): bash tools/build_lib_at.sh COMMIT OUT.so   (e.g. 28e5c00 tools/bin/lib_r03.so)
# Newer ABI entries the control lacks are stubbed so gaplac_amd/_native.py can bind it.
set -e
C=$1; OUT=$(readlink -f "$2")
T=$(mktemp -d)
mkdir -p $T/gaplac_amd/csrc $T/include
for f in gaplac_kernels.hip gaplac_api.hip gaplac_dist.hip gaplac_internal.h; do git show $C:gaplac_amd/csrc/$f > $T/gaplac_amd/csrc/$f; done
git show $C:include/gaplac.h > $T/include/gaplac.h
STUBS=""
grep -q gaplac_ctx_release $T/include/gaplac.h || STUBS="$STUBS extern \"C\" int gaplac_ctx_release(gaplac_ctx*) { return 0; }"
printf '#include "gaplac_internal.h"\n%s\n' "$STUBS" > $T/gaplac_amd/csrc/stubs.hip
cd $T/gaplac_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o "$OUT" gaplac_kernels.hip gaplac_api.hip gaplac_dist.hip stubs.hip
rm -rf $T
echo "$OUT"
