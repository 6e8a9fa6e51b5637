#!/bin/bash
# Build a compile-time variant of libpt.so into build_variants/NAME/libpt.so (CPU side, before a
# gpurun A/B):   tools/build_variant.sh NAME "-DPT_SECPROF ..." ['sed expression applied to csrc/*']
# (the tuned constants are constexprs: e.g. 's/kGoutLdsGltf = 4/kGoutLdsGltf = 0/')
# The in-tree libpt.so is untouched; tools/gpu_bench_*.sh / gpu_variants.sh pick the variants up.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; FLAGS=$2
OUT=$ROOT/build_variants/$NAME
rm -rf "$OUT"; mkdir -p "$OUT/pkg" "$OUT/include"
cp -r "$ROOT/babylon.js-pathtracing-renderer_amd/csrc" "$ROOT/babylon.js-pathtracing-renderer_amd/Makefile" "$OUT/pkg/"
cp "$ROOT/include/pt.h" "$OUT/include/"
if [ -n "$3" ]; then sed -i "$3" "$OUT"/pkg/csrc/*.h "$OUT"/pkg/csrc/*.hip "$OUT"/pkg/csrc/*.cpp; fi
if [ -n "$4" ]; then python3 "$4" "$OUT/pkg/csrc" $5; fi
make -s -C "$OUT/pkg" -j8 libpt.so \
  HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wno-unused-function -Wno-unused-result -Wno-unused-value $FLAGS" >/dev/null
mv "$OUT/pkg/libpt.so" "$OUT/libpt.so"
rm -rf "$OUT/pkg" "$OUT/include"
echo "built $OUT/libpt.so ($FLAGS)"
