#!/bin/bash
# Diagnostic builds of libgymchess.so with alternative compiler options (tools/_lib_<tag>.so;
# compared on the GPU with tools/ab_lib.py).  Usage: tools/build_variants.sh tag "flags" ...
cd "$(dirname "$0")/.."
SRC=gym-chess_amd/csrc/gymchess.hip
while [ $# -ge 2 ]; do
  tag=$1; flags=$2; shift 2
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -mllvm -amdgpu-kernarg-preload-count=16 $flags \
        -o tools/_lib_$tag.so $SRC &
done
wait
ls -la tools/_lib_*.so
