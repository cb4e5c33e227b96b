#!/bin/bash
# tools/isa_diff.sh REV [KERNEL...] -- compare the gfx950 ISA of the product
# kernels built from git revision REV with the working tree's (hygiene
# changes must leave the default build's machine code unchanged).  Prints
# one line per kernel: same / DIFF (instruction counts).
set -e
REV=${1:?rev}; shift
KERNELS=${@:-fd_k_prep fd_k_front fd_k_decomp fd_k_dsm fd_k_dsm_setup fd_k_dsm_pool fd_k_dsm_final fd_k_dsm_quad fd_k_dsm_oct fd_k_sha512_batch}
T=$(mktemp -d)
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $T/old/firedancer_amd/csrc $T/old/include
for f in $(git -C $ROOT ls-tree --name-only $REV firedancer_amd/csrc/ include/); do git -C $ROOT show $REV:$f > $T/old/$f; done
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -Wno-unused-result -Wno-unused-value --cuda-device-only -S"
/opt/rocm/bin/hipcc $FLAGS -I$T/old/include -I$T/old/firedancer_amd/csrc $T/old/firedancer_amd/csrc/fd_ed25519_gpu_kernels.hip -o $T/old.s 2>/dev/null
/opt/rocm/bin/hipcc $FLAGS -I$ROOT/include -I$ROOT/firedancer_amd/csrc $ROOT/firedancer_amd/csrc/fd_ed25519_gpu_kernels.hip -o $T/new.s 2>/dev/null
body() { awk -v k="$2" '$0 ~ "^"k":" {on=1; next} on && /^\.Lfunc_end/ {exit} on && /^[ \t]+(s_|v_|global_|ds_|buffer_|flat_)/ {gsub(/;.*/,""); print}' $1; }
for k in $KERNELS; do
  body $T/old.s $k > $T/o.txt; body $T/new.s $k > $T/n.txt
  if cmp -s $T/o.txt $T/n.txt; then echo "$k same ($(wc -l < $T/n.txt) instructions)"; else echo "$k DIFF ($(wc -l < $T/o.txt) -> $(wc -l < $T/n.txt))"; fi
done
[ -n "$KEEP" ] && echo "kept $T" || rm -rf $T
