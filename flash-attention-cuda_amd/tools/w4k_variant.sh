#!/bin/bash
# Build an experiment variant of the library with a differently generated
# short-tier segment program: tools/w4k_variant.sh NAME "W4K_XP=a,b" ->
# lib/libfa_mi355x_NAME.so (generated into a temporary include directory;
# the product csrc/fa_w4k_item.inc is never touched)
set -e
cd "$(dirname "$0")/.."
name=$1; envs=$2; DEFS=$3
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
env -u W4_DIAG -u W4_XP -u W4K_XP -u W4K_V_AHEAD -u W4K_DIAG $envs python3 csrc/gen_w4k_item.py "$tmp/fa_w4k_item.inc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-honor-nans -I"$tmp" -I../include -Icsrc \
  $DEFS -shared csrc/fa_fwd.hip csrc/flash_attention_v9.cpp -o lib/libfa_mi355x_$name.so
