#!/bin/bash
# A/B against committed kernels: scripts/build_ref_variant.sh <tag> <git-ref> [extra hipcc flags...]
# builds csrc/kernels as of <git-ref> into serverless_learn_amd/_native/variants/libslkernels_<tag>.so
# (load with SL_KERNELS_SO=..., or "gpu_task.sh ab <reps> base,<tag>").  Runs here, on the CPU.
set -e
tag=$1; ref=$2; shift 2
src=build/refsrc/$tag
rm -rf $src && mkdir -p $src
git archive "$ref" csrc/kernels | tar -x -C $src
out=serverless_learn_amd/_native/variants
mkdir -p $out build/variants/$tag
objs=""
for f in $src/csrc/kernels/*.hip; do
  o=build/variants/$tag/$(basename $f).o
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$src/csrc/kernels -munsafe-fp-atomics -Wno-unused-result "$@" -c $f -o $o &
  objs="$objs $o"
done
wait
hipcc --offload-arch=gfx950 -shared -fPIC $objs -o $out/libslkernels_$tag.so
echo $out/libslkernels_$tag.so
