#!/usr/bin/env bash
# Kernel levels on the GPU box: bench.py at C3 (and C2) for each specialisation / edit the drop-in
# can meet, one JSON line each (gpurun_out/TAG_level_NAME.json); scripts/levels_summary.py TAG
# collects them into profiles/TAG_kernel_levels_c3.json with each level's ratio to the literal kernel.
#   LEVELS="c3 c3_tilted ..." selects levels (default: all below).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r06}
declare -A ARGS=(
  [c3]=""
  [c3_refleaks]="--reference-leaks"
  [c3_tilted]="--camera tilted"
  [c3_light]="--light-y 81.4"
  [c3_light_tilted]="--light-y 81.4 --camera tilted"
  [c3_light_grow]="--light-y 81.0 --light-grow 1"
  [c3_movebox]="--move-box 1"
  [c3_room]="--room-depth 171"
  [c3_room160]="--room-depth 160"
  [c3_movebox_cornell]="--move-box 1 --kernel-level const"
  [c3_const]="--kernel-level const"
  [c3_cornell]="--kernel-level cornell"
  [c3_generic]="--kernel-level generic"
  [c2]="--config c2"
  [c2_tilted]="--config c2 --camera tilted"
  [c2_light]="--config c2 --light-y 81.4"
)
ORDER="c3 c3_tilted c3_light c3_light_tilted c3_light_grow c3_movebox c3_room c3_room160 c3_refleaks c3_movebox_cornell c3_const c3_cornell c3_generic c2 c2_tilted c2_light"
for name in ${LEVELS:-$ORDER}; do
  timeout -k 10 240 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline ${ARGS[$name]} \
    > gpurun_out/${TAG}_level_$name.json 2> gpurun_out/${TAG}_level_$name.err
  rc=$?; echo "level $name exit $rc"; [ $rc -eq 0 ] || exit $rc
done
