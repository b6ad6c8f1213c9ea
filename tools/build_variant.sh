#!/bin/bash
# Build a variant of libsfmcore.so with extra compile flags on one source:
#   tools/build_variant.sh OUT.so SOURCE.hip [flags...]
# (the other objects come from build/, made by `make`)
set -e
out=$1; src=$2; shift 2
base=$(basename "$src")
mkdir -p build_var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mcode-object-version=5 -Wall -Wno-unused-result \
    -I/opt/rocm/include "$@" -c "$src" -o "build_var/$base.o"
objs=$(ls build/*.o | grep -v "/$base.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out" $objs "build_var/$base.o" -ldl
