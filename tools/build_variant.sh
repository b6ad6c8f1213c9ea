#!/bin/bash
# A/B builds of libsfmcore.so: tools/build_variant.sh NAME SOURCE "EXTRA HIPCC FLAGS"
# Rebuilds one csrc/ source with extra flags and links it with the regular
# objects into build/var_NAME/libsfmcore.so (load with SFMCORE_LIB=...).
set -e
cd "$(dirname "$0")/.."
make -s 3dreconstruction_amd/lib/libsfmcore.so
NAME=$1; SRC=$2; FLAGS=$3
D=build/var_$NAME
mkdir -p $D
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mcode-object-version=5 -I/opt/rocm/include $FLAGS \
    -c 3dreconstruction_amd/csrc/$SRC -o $D/$SRC.o
OBJS=$(ls build/*.hip.o build/*.cpp.o | grep -v "/$SRC.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libsfmcore.so $OBJS $D/$SRC.o -ldl
echo $D/libsfmcore.so
