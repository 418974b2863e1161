#!/bin/bash
# Build engine variants (compile-time knobs) as tools/micro/variants/libpcgpu_<name>.so for
# tools/variant_bench.sh. usage: tools/build_variants.sh name1 "-DKNOB=1 ..." name2 "..." ...
set -eu
cd "$(dirname "$0")/../rcaeval_amd/csrc"
mkdir -p ../../tools/micro/variants
rm -f ../../tools/micro/variants/libpcgpu_*.so
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  make -s -j8 BUILD=/tmp/pcg_build_$name OUT=../../tools/micro/variants/libpcgpu_$name.so EXTRA="$flags"
  echo "built $name ($flags)"
done
