#!/bin/bash
# Build a same-box A/B variant of liblbwn.so into lb-wavenet_amd/lbwn/abl/liblbwn_g<NAME>.so: the
# current objects with the listed sources taken from a git revision.
# Usage: bash tools/build_variant.sh NAME REV file.hip [file.hip|file.h ...]   (files relative to csrc/)
set -e
NAME=$1; REV=$2; shift 2
cd "$(dirname "$0")/../lb-wavenet_amd/csrc"
make -s -j8 ARCH=gfx950 >/dev/null
mkdir -p ../lbwn/abl build/var_$NAME
# headers listed (e.g. prologue.h) are taken from REV too: a quoted #include finds them beside the
# variant sources before -I.
for h in "$@"; do
  [ "${h##*.}" = h ] && git show $REV:lb-wavenet_amd/csrc/$h > build/var_$NAME/$h
done
OBJS=""
for f in gemm layer misc gen cond engine capi; do
  src=$f.hip; [ -f $src ] || src=$f.cpp
  if [[ " $* " == *" $src "* ]]; then
    git show $REV:lb-wavenet_amd/csrc/$src > build/var_$NAME/$src
    X=""; [ "${src##*.}" = cpp ] && X="-x hip"
    F=""; [ $f = gemm ] && F="-fno-slp-vectorize"
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $F -I. $X -c build/var_$NAME/$src -o build/var_$NAME/$f.o
    OBJS="$OBJS build/var_$NAME/$f.o"
  else
    OBJS="$OBJS build/$f.o"
  fi
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC $OBJS -o ../lbwn/abl/liblbwn_g$NAME.so
echo built ../lbwn/abl/liblbwn_g$NAME.so
