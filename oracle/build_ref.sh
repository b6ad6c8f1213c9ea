#!/bin/bash
# Build the golden-descriptor tool from the reference's own VLFeat C sources
# where they lie (read-only), outputs only into oracle/_ref/.  Test
# infrastructure: nothing in the product links or loads it.
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
VL=/root/reference/src/nonFree/sift/vl
OUT="$HERE/_ref"
if [ ! -d "$VL" ]; then echo "reference VLFeat not present; skipping"; exit 0; fi
mkdir -p "$OUT"
SRC="$VL/generic.c $VL/host.c $VL/imopv.c $VL/imopv_sse2.c $VL/mathop.c $VL/mathop_sse2.c $VL/random.c $VL/sift.c"
gcc -O2 -std=gnu99 -DVL_DISABLE_THREADS -DVL_DISABLE_SSE2 -I"$VL" -o "$OUT/vlsift_tool" \
    "$HERE/vlsift_tool.c" $SRC -lm 2> "$OUT/build.log" || { cat "$OUT/build.log"; exit 1; }
echo "built $OUT/vlsift_tool"
