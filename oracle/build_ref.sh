#!/usr/bin/env bash
# Build the *reference* smallpt (maurock/small-pathtracer HEAD) as a test oracle.
#
# TEST INFRASTRUCTURE ONLY. Compiles /root/reference/src/smallpt.cpp where it lies,
# streaming it through sed (the patch recipe of SURVEY.md Appendix A) straight into
# g++ via stdin: no reference source is copied into this repository or anywhere on
# disk. Outputs go only to oracle/_ref/ (git-ignored).
#
# Patch (line numbers of /root/reference/src/smallpt.cpp):
#   :424-442  delete the Q-learning early return -> the live path tracer at :444-480 runs
#   :503      srand(time(NULL)) -> srand(seed), seed = argv[4] (default 1)
#   :507-508  w, h, samps from argv[1..3]
#   :517      skip create_state_space (keeps the rand() stream starting at the pixel loop)
#   :548      output file name from argv[5]
#   :464      (cosine variant only) q < 1  ->  q < 0
#   :340-360  (uniform variant only) cosine body out, the commented uniform hemisphere body in
# Pinned build: g++ -O3, x86-64 baseline (no -march=native: FMA contraction changes bits).
set -euo pipefail
REF=${REF:-/root/reference/src}
OUT=${OUT:-$(cd "$(dirname "$0")" && pwd)/_ref}
if [ ! -f "$REF/smallpt.cpp" ]; then
  echo "reference not present at $REF; skipping oracle/_ref build" >&2
  exit 0
fi
mkdir -p "$OUT"
common_sed=(
  -e '424,442d'
  -e '503s/srand(time(NULL));/int seed_ = argc > 4 ? atoi(argv[4]) : 1; srand(seed_);/'
  -e '507s/int w = 512, h = 512;/int w = argc > 1 ? atoi(argv[1]) : 512, h = argc > 2 ? atoi(argv[2]) : 512;/'
  -e '508s/int samps = 16;/int samps = argc > 3 ? atoi(argv[3]) : 16;/'
  -e '517s/create_state_space(dict)/0/'
  -e '548s/"show_allrect_differentplane_red_state.ppm"/(argc > 5 ? argv[5] : "out.ppm")/'
)
build() {  # $1 = output binary, rest = extra sed expressions
  local bin=$1; shift
  sed "${common_sed[@]}" "$@" "$REF/smallpt.cpp" \
    | g++ -O3 -w -x c++ -I"$REF" - -o "$OUT/$bin"
}
build smallpt_nee
build smallpt_cos -e '464s/if (q < 1)/if (q < 0)/'
# uniform-hemisphere variant of random_scattering: the live cosine body :340-347 removed and the
# commented-out uniform body :352-359 enabled (its /* and */ lines :351, :360 removed)
build smallpt_uni -e '340,347d' -e '351d' -e '360d'
# statistics-only variant (tests/test_fidelity.py): the per-row erand48 state {0,0,y^3} of :530
# does not depend on the seed, so every scattering/RR draw repeats across seeds and only rand()
# (jitter, light point, Q) varies. Seeding the middle word with the seed gives independent runs.
xs='530s/Xi\[3\] = { 0, 0, y \* y \* y }/Xi[3] = { 0, (unsigned short)seed_, (unsigned short)(y * y * y) }/'
build smallpt_nee_xs -e "$xs"
build smallpt_cos_xs -e '464s/if (q < 1)/if (q < 0)/' -e "$xs"
build smallpt_uni_xs -e '340,347d' -e '351d' -e '360d' -e "$xs"
# the reference's own OpenMP loop (bench.py cpu_baseline): the pragma
# :526 uncommented and the row loop :528 made canonical (i = y*w per row). rand() stays the
# global, locked libc generator, as the reference would run it.
omp=(-e '526s|// #pragma omp parallel for|#pragma omp parallel for|'
     -e '528s/for (int y = 0, i = 0; y < h; y++) {/for (int y = 0; y < h; y++) { int i = y * w;/')
buildomp() {
  local bin=$1; shift
  sed "${common_sed[@]}" "$@" "$REF/smallpt.cpp" \
    | g++ -O3 -fopenmp -w -x c++ -I"$REF" - -o "$OUT/$bin"
}
buildomp smallpt_nee_omp "${omp[@]}"
buildomp smallpt_cos_omp -e '464s/if (q < 1)/if (q < 0)/' "${omp[@]}"
echo "built $OUT/smallpt_{nee,cos,uni} $OUT/smallpt_{nee,cos,uni}_xs $OUT/smallpt_{nee,cos}_omp"
