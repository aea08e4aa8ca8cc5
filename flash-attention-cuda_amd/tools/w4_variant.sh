#!/bin/bash
# Build a diagnostic / experiment variant of the library with a differently
# generated W4 item program:  tools/w4_variant.sh NAME "W4_DIAG=stamps W4_XP=a,b"
# -> lib/libfa_mi355x_NAME.so.  The variant's item programs (W4 and W4P) are
# generated into a temporary directory placed first on the include path, so the
# product csrc/fa_w4_item.inc / fa_w4p_item.inc are never touched.
set -e
cd "$(dirname "$0")/.."
name=$1; envs=$2
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
# every exported W4*/W4P* knob is stripped first (an exported knob would
# otherwise leak into every variant build), then only $envs applied
clean=$(env | sed -n 's/^\(W4[A-Z0-9_]*\)=.*/-u \1/p' | tr '\n' ' ')
env $clean $envs python3 csrc/gen_w4_item.py "$tmp/fa_w4_item.inc"
env $clean $envs python3 csrc/gen_w4p_item.py "$tmp/fa_w4p_item.inc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-honor-nans ${W4_HIPFLAGS:-} -I"$tmp" -I../include -Icsrc \
  -shared csrc/fa_fwd.hip csrc/flash_attention_v9.cpp -o lib/libfa_mi355x_$name.so
