#!/bin/bash
# Build the kernel library of another git revision into ab/libssamd_kernels_<rev>.so for same-box
# A/B timing (SSAMD_KERNEL_LIB=ab/... python bench.py ...).  Usage: tools/build_ab.sh <rev>
set -euo pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
rev=$(git -C "$R" rev-parse --short "$1")
src=$(mktemp -d /tmp/ab_src.XXXX)
git -C "$R" archive "$rev" csrc | tar -x -C "$src"
mkdir -p "$R/ab"
objs=()
for f in "$src"/csrc/*.hip; do
  o="$src/$(basename "$f").o"
  /opt/rocm/bin/hipcc -c "$f" -o "$o" --offload-arch=gfx950 -std=c++17 -fPIC -Wno-unused-function \
    -Wno-unused-variable -munsafe-fp-atomics -I "$src/csrc" -O3 &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$R/ab/libssamd_kernels_$rev.so" "${objs[@]}"
rm -rf "$src"
echo "$R/ab/libssamd_kernels_$rev.so"
