#!/bin/bash
# Link an A/B build of librmd.so with one source recompiled under -D knobs.
# usage: tools/build_variant.sh NAME SOURCE.hip "-DKNOB=V ..."  -> tools/_ab/librmd_NAME.so
set -e
cd "$(dirname "$0")/../raft-meets-dicl_amd/csrc"
make -s -j8 >/dev/null
NAME=$1; SRC=$2; DEFS=$3
mkdir -p build/var ../../tools/_ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -fno-slp-vectorize \
    -I../../include -I. $DEFS -c $SRC -o build/var/${SRC%.hip}_$NAME.o
OBJS=$(ls build/*.o | grep -v "build/${SRC%.hip}.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/_ab/librmd_$NAME.so $OBJS build/var/${SRC%.hip}_$NAME.o
echo tools/_ab/librmd_$NAME.so
