#!/bin/bash
# Build a diagnostic / experiment variant of the library with a differently
# generated W4 item program:  tools/w4_variant.sh NAME "W4_DIAG=stamps W4_XP=a,b"
# -> lib/libfa_mi355x_NAME.so  (the product fa_w4_item.inc is regenerated after)
set -e
cd "$(dirname "$0")/.."
name=$1; envs=$2
env $envs python3 csrc/gen_w4_item.py csrc/fa_w4_item.inc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-honor-nans -I../include -Icsrc \
  -shared csrc/fa_fwd.hip csrc/flash_attention_v9.cpp -o lib/libfa_mi355x_$name.so
python3 csrc/gen_w4_item.py csrc/fa_w4_item.inc
