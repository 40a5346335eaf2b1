#!/bin/bash
# Kernel A/B experiments: build a self-contained copy of the package whose throughput kernel comes
# from an alternative source file.  usage: tools/build_variant.sh NAME path/to/variant.hip [HDR_DIR] [OBJ]
# HDR_DIR (optional, "" for none): directory whose device headers (device_math.h, kernels.h) the
# variant uses.  OBJ (optional): the object the variant replaces (default pbs_kernels; br_quad, br_wide).
# EXTRA_FLAGS (env, optional): extra compiler flags for the variant object.
# Output: build_variants/NAME/{fhe_sign,lib/libfhe_rocm.so} (git-ignored); the regular objects of
# the other sources are reused from fhe-sign_amd/build.  Run with tools/variant_probe.py.
set -e
NAME=$1; SRC=$2; HDR=${3:-}; OBJ=${4:-pbs_kernels}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/fhe-sign_amd
OUT=$ROOT/build_variants/$NAME
make -s -C $PKG
mkdir -p $OUT/lib $OUT/obj
if [ -n "$HDR" ]; then
  VS=$HDR/_variant_$NAME.hip
else
  VS=$PKG/csrc/_variant_$NAME.hip
fi
cp "$SRC" $VS
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off ${EXTRA_FLAGS:-} -I$ROOT/include ${HDR:+-I$HDR} -I$PKG/csrc --offload-arch=gfx950 \
    -c -o $OUT/obj/$OBJ.o $VS
rm -f $VS
OBJS=$(ls $PKG/build/*.o | grep -v "/$OBJ.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT/lib/libfhe_rocm.so $OUT/obj/$OBJ.o $OBJS -lpthread -L/opt/rocm/lib -lrccl
rm -rf $OUT/fhe_sign && cp -r $PKG/fhe_sign $OUT/fhe_sign
echo "built $OUT"
