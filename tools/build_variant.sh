#!/bin/bash
# Build a tuning variant of libcordagpu.so into abvar/libcg_<name>.so, reusing the
# in-tree objects for every source but the ones listed in $SRCS (default: the Ed25519
# kernels):  bash tools/build_variant.sh <name> -DKNOB=value ...
set -e
name=${1:?name}; shift
cd "$(dirname "$0")/../corda_amd/csrc"
srcs=${SRCS:-ed25519_kernels}
rm -rf build_$name && mkdir -p build_$name && cp build/*.o build_$name/
for s in $srcs; do rm -f build_$name/$s.o; done
make -s BUILD=build_$name OUT=../../abvar/libcg_$name.so EXTRA="$*" ../../abvar/libcg_$name.so
rm -rf build_$name
echo "abvar/libcg_$name.so"
