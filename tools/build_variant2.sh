#!/bin/bash
# Build a variant of libsfmcore.so with extra compile flags on SEVERAL sources
# (e.g. a ba_types.h macro read by both the planner and the kernels):
#   tools/build_variant2.sh OUT.so "SRC1 SRC2 ..." [flags...]
set -e
out=$1; srcs=$2; shift 2
mkdir -p build_var
skip=""
objs_var=""
for src in $srcs; do
    base=$(basename "$src")
    x=""; [[ "$src" == *.cpp ]] && x="-fvisibility=hidden -fvisibility-inlines-hidden -x hip"
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mcode-object-version=5 -Wall -Wno-unused-result \
        -I/opt/rocm/include $x "$@" -c "$src" -o "build_var/$base.o"
    skip="$skip|/$base.o\$"
    objs_var="$objs_var build_var/$base.o"
done
objs=$(ls build/*.o | grep -Ev "${skip#|}")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out" $objs $objs_var -ldl
