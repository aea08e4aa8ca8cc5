#!/bin/bash
# Build a diagnostic / experiment variant of the library with a differently
# generated W4 item program:  tools/w4_variant.sh NAME "W4_DIAG=stamps W4_XP=a,b"
# -> lib/libfa_mi355x_NAME.so.  The variant's item program is generated into a
# temporary directory placed first on the include path, so the product
# csrc/fa_w4_item.inc is never touched.
set -e
cd "$(dirname "$0")/.."
name=$1; envs=$2
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
env -u W4_DIAG -u W4_XP -u W4_OPOL -u W4_WAGE -u W4_V_AHEAD -u W4_MAX_OFF -u W4_LEFT_OFF -u W4_DMA_AT -u W4_DMA_SP $envs python3 csrc/gen_w4_item.py "$tmp/fa_w4_item.inc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-honor-nans ${W4_HIPFLAGS:-} -I"$tmp" -I../include -Icsrc \
  -shared csrc/fa_fwd.hip csrc/flash_attention_v9.cpp -o lib/libfa_mi355x_$name.so
