#!/bin/bash
# Disassemble the gfx950 code object embedded in a libdrt build: tools/disasm.sh LIB.so OUT.dis
set -e
B=/opt/rocm/lib/llvm/bin
tmp=$(mktemp -d)
objcopy -O binary --only-section=.hip_fatbin "$1" $tmp/fb.bin
$B/clang-offload-bundler --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input=$tmp/fb.bin \
    --output=$tmp/k.co --unbundle
$B/llvm-objdump -d --no-show-raw-insn $tmp/k.co > "$2"
rm -rf $tmp
