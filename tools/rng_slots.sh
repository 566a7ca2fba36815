#!/usr/bin/env bash
# Static VALU issue slots of the per-vertex random words per candidate generator (tools/rng_slots.hip),
# each net of the empty kernel's load/store slots. CPU only (ISA listing).
set -e
cd "$(dirname "$0")/.."
mkdir -p build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --offload-device-only -S -o build/rng_slots.s tools/rng_slots.hip
base=$(python tools/isa_blocks.py build/rng_slots.s "k_empty:" | head -1 | sed -E "s/.*'slots': ([0-9]+).*/\1/")
for k in k_philox k_lcg48 k_lcg48_steps k_pcg32 k_xs32; do
  s=$(python tools/isa_blocks.py build/rng_slots.s "$k:" | head -1 | sed -E "s/.*'slots': ([0-9]+).*/\1/")
  echo "$k $((s - base))"
done
