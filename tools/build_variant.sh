#!/bin/bash
# Kernel A/B experiments: build a self-contained copy of the package whose throughput kernel comes
# from an alternative source file.  usage: tools/build_variant.sh NAME path/to/pbs_kernels_variant.hip [HDR_DIR]
# HDR_DIR (optional): directory whose device headers (device_math.h, kernels.h) the variant uses.
# Output: build_variants/NAME/{fhe_sign,lib/libfhe_rocm.so} (git-ignored); the regular objects of
# the other sources are reused from fhe-sign_amd/build.  Run with tools/variant_probe.py.
set -e
NAME=$1; SRC=$2; HDR=${3:-}
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
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -I$ROOT/include ${HDR:+-I$HDR} -I$PKG/csrc --offload-arch=gfx950 \
    -c -o $OUT/obj/pbs_kernels.o $VS
rm -f $VS
OBJS=$(ls $PKG/build/*.o | grep -v pbs_kernels.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT/lib/libfhe_rocm.so $OUT/obj/pbs_kernels.o $OBJS -lpthread -L/opt/rocm/lib -lrccl
rm -rf $OUT/fhe_sign && cp -r $PKG/fhe_sign $OUT/fhe_sign
echo "built $OUT"
