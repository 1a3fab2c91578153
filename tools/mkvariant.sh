#!/bin/bash
# Build an A/B variant of libcfws.so: the translation units named in $UNITS
# (default cfws_uniform) recompiled with extra flags, linked with the
# in-tree objects of the others (run `make` first).
#   tools/mkvariant.sh <name> "<-D flags>"   -> build/variants/libcfws_<name>.so
set -e
cd "$(dirname "$0")/.."
name=$1; flags=$2
D=build/variants/$name; mkdir -p "$D"
objs=""
for o in build/cfws_*.o; do
  u=$(basename "$o" .o)
  if [[ " ${UNITS:-cfws_uniform} " == *" $u "* ]]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Iinclude \
        -Icoldforce_amd/csrc $flags -c coldforce_amd/csrc/$u.hip -o "$D/$u.o"
    objs="$objs $D/$u.o"
  else
    objs="$objs $o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/variants/libcfws_$name.so $objs
echo "build/variants/libcfws_$name.so"
