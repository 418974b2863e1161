#!/bin/bash
# Build engine variants (compile-time knobs) as tools/ab/libpcgpu_<name>.so for
# tools/variant_bench.sh. usage: tools/build_variants.sh name1 "-DKNOB=1 ..." name2 "..." ...
set -eu
cd "$(dirname "$0")/../rcaeval_amd/csrc"
mkdir -p ../../tools/ab
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  make -s -j8 BUILD=/tmp/pcg_build_$name OUT=../../tools/ab/libpcgpu_$name.so EXTRA="$flags"
  echo "built $name ($flags)"
done
