#!/bin/bash
# An alternative libcome.so for A/B runs (scripts/ab.sh "name:COME_LIB_PATH=..."): the product
# objects from csrc/build with ONE source recompiled with extra flags.
#   bash scripts/build_ab.sh NAME SOURCE "-DFLAG=1 ..."   -> csrc/build/ab/libcome_NAME.so
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
C="$ROOT/nodeembedding-to-communityembedding_amd/csrc"
NAME=$1; SRC=$2; FLAGS=$3
make -s -C "$C" -j8
mkdir -p "$C/build/ab/$NAME"
OBJ="$C/build/ab/$NAME/$(basename "${SRC%.*}").o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall \
  -I"$ROOT/include" $FLAGS -c "$C/$SRC" -o "$OBJ"
OBJS=$(ls "$C"/build/*.o | grep -v "/$(basename "${SRC%.*}").o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$C/build/ab/libcome_$NAME.so" $OBJS "$OBJ" -pthread
echo "$C/build/ab/libcome_$NAME.so"
