#!/bin/bash
# A/B kernel builds: scripts/build_variant.sh <tag> <extra hipcc flags...>
# -> serverless_learn_amd/_native/variants/libslkernels_<tag>.so (load with SL_KERNELS_SO=...)
set -e
tag=$1; shift
out=serverless_learn_amd/_native/variants
mkdir -p $out build/variants/$tag
objs=""
for f in csrc/kernels/*.hip; do
  o=build/variants/$tag/$(basename $f).o
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Icsrc/kernels -munsafe-fp-atomics -Wno-unused-result "$@" -c $f -o $o &
  objs="$objs $o"
done
wait
hipcc --offload-arch=gfx950 -shared -fPIC $objs -o $out/libslkernels_$tag.so
if nm -D --undefined-only $out/libslkernels_$tag.so | grep -q __device_stub__; then
  echo "undefined kernel launch stubs in $out/libslkernels_$tag.so" >&2; exit 1
fi
echo $out/libslkernels_$tag.so
