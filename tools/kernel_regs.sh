#!/bin/bash
# kernel_regs.sh OBJ [PATTERN] -- VGPR count and spill count of every kernel in
# a built object's gfx950 code object (no recompile): build/kernels_p4.o etc.
set -e
obj=$1; pat=${2:-.}
tmp=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section .hip_fatbin=$tmp/fb "$obj" $tmp/copy.o
/opt/rocm/lib/llvm/bin/clang-offload-bundler --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 \
  --input=$tmp/fb --output=$tmp/co --unbundle
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $tmp/co | grep -E "\.name:|vgpr_spill_count|\.vgpr_count" | paste - - - |
  awk '{print $2, "vgpr", $4, "spill", $6}' | grep -E "$pat" || true
rm -rf $tmp
