#!/usr/bin/env bash
# Resource usage (VGPRs / spills / occupancy) of the render kernels: tools/vgprs.sh [extra hipcc flags]
cd "$(dirname "$0")/../small-pathtracer_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize --offload-device-only -S \
  -o /tmp/vgprs.s spt_kernel.hip -Rpass-analysis=kernel-resource-usage "$@" 2>&1 |
  grep -E "Function Name|    VGPRs:|TotalSGPRs|Occupancy|Spill" | sed 's/ \[-Rpass.*//; s/.*remark: *//' |
  paste - - - - - - | grep render_kernel | sed 's/Function Name: _ZN3spt13render_kernelINS_4Topo//'
