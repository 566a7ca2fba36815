#!/usr/bin/env bash
# Build A/B library variants into build/ab/<name>.so: scripts/build_variants.sh name:"-DFLAG ..." ...
set -eu
cd "$(dirname "$0")/../small-pathtracer_amd/csrc"
mkdir -p ../../build/ab
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -Wall -Wno-unused-result"
pids=()
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  /opt/rocm/bin/hipcc $FLAGS $defs -shared -o ../../build/ab/$name.so spt_kernel.hip spt_image.hip spt_multi.hip spt_host.cpp -lrccl &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
ls -la ../../build/ab
