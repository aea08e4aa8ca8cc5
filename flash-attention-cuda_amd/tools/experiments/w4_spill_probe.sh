#!/bin/bash
# Register report (VGPR/AGPR/spills) and v_accvgpr copy count of the W4 probe
# kernels -- the evidence that hipcc cannot hold 64 query rows per wave
# (DESIGN.md section 3).  CPU only.
cd "$(dirname "$0")/../.." || exit 1
out=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-honor-nans -Icsrc -I../include \
  --cuda-device-only -S tools/experiments/w4_spill_probe.hip -o "$out/w4.s" \
  -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs:|AGPRs:|VGPRs Spill|ScratchSize" | sed 's/.*remark: *//; s/ \[-Rpass.*//'
echo "v_accvgpr instructions: $(grep -c v_accvgpr "$out/w4.s"), v_mfma: $(grep -c v_mfma "$out/w4.s")"
rm -rf "$out"
