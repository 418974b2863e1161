#!/bin/bash
# Build an A/B variant of libpcgpu.so with extra -D flags on skeleton.hip only (the other objects
# are the in-tree build's): tools/build_variant.sh NAME "-DPCG_X=1 -DPCG_Y=2"
# -> tools/ab/libpcgpu_NAME.so (+ its kernel resource report)
set -eu
cd "$(dirname "$0")/../rcaeval_amd/csrc"
name=$1; flags=$2
out=../../tools/ab
mkdir -p $out build
make -s -j8 >/dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../../include -I. -Wall -Wno-unused-result \
  -Wno-unused-value $flags -c skeleton.hip -o build/skeleton_$name.o -Rpass-analysis=kernel-resource-usage \
  2> $out/$name.resources.txt
objs=$(ls build/*.o | grep -v "skeleton_" | grep -v "build/skeleton.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libpcgpu_$name.so build/skeleton_$name.o $objs -ldl
rm build/skeleton_$name.o
echo "built $out/libpcgpu_$name.so"
