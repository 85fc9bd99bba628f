#!/usr/bin/env bash
# Build the gfx950 kernel library of a git revision into ab/lib<name>.so for same-box A/B runs:
#   bash scripts/dev/build_ab.sh HEAD head && RAFIKI_KERNEL_LIB=ab/libhead.so python bench.py
set -euo pipefail
rev=${1:?rev}; name=${2:?name}
root=$(cd "$(dirname "$0")/.." && pwd)
work=$(mktemp -d)
git -C "$root" archive "$rev" csrc/kernels | tar -x -C "$work"
mkdir -p "$root/ab"
objs=()
for s in "$work"/csrc/kernels/*.hip; do
  o="$work/$(basename "$s" .hip).o"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -c "$s" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "${objs[@]}" -o "$root/ab/lib$name.so"
rm -rf "$work"
echo "$root/ab/lib$name.so"
