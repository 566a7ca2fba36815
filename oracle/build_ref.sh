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
#   :464      (Q = 0.5 variant) q < 1  ->  q < 0.5
#   :19, :254, :295-310, :447  (sphere variants) see below
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
# NEE-mix probability Q = 0.5 (:464 `q < 1` -> `q < 0.5`: half light sampling, half cosine; the
# estimator of the shipped image_32pps_halflighthalfimportance.ppm lineage)
build smallpt_q05 -e '464s/if (q < 1)/if (q < 0.5)/'
build smallpt_q05_xs -e '464s/if (q < 1)/if (q < 0.5)/' -e "$xs"
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

# Config 5's 32-sphere scene rendered by the reference's OWN Sphere class (:223-254, fp64,
# eps 1e-4) and its own radiance/intersect ("replace the rect[] initialiser
# :287-311 with the 32-sphere scene using the reference's own Sphere class"):
#   :19       NUMBER_OBJ 17 -> 39
#   :295-310  the two boxes out; after the light (:294) the 32 spheres of spt_scene_spheres32
#             (r = 6 at x = 1 + 98 (col + .5) / 8, y = 6, z = 30 + 30 row, colour pal[(3 row + col) % 8]),
#             written with the same double expressions as small-pathtracer_amd/csrc/spt_host.cpp
#   :254      Sphere gets the two Q-learning methods of the Hitable interface (:87-88), which it
#             lacks (it would be abstract). They are never called: create_state_space is skipped
#             (:517), and the methods return zeros.
#   :447      (depth-capped variants) `if (depth + 1 >= D) return hit.e;` before the RR line :448:
#             the path ends at vertex depth D with the hit's emission (spt_params.max_depth = D)
sph_sed="$OUT/spheres32.sed"
{
  echo '19s/NUMBER_OBJ = 17;/NUMBER_OBJ = 39;/'
  echo '254i\'
  echo '	std::array<float, 3> add_key(Vec \&) const { return {0, 0, 0}; } std::array<float, 3> add_value(std::array<float, 3> \&) const { return {0, 0, 0}; }'
  echo '295,310d'
  echo '294a\'
  pal=('.75, .25, .25' '.25, .75, .25' '.25, .25, .75' '.75, .75, .25' '.25, .75, .75' '.75, .25, .75' '.9, .9, .9' '.6, .45, .3')
  for row in 0 1 2 3; do
    for col in 0 1 2 3 4 5 6 7; do
      sep=','; [ "$row$col" = 37 ] && sep=''
      line="	new Sphere(6.0, Vec(1.0 + 98.0 * ($col + 0.5) / 8.0, 6.0, 30.0 + 30.0 * $row), Vec(), Vec(${pal[$(( (row * 3 + col) % 8 ))]}), DIFF)$sep"
      [ "$row$col" = 37 ] && echo "$line" || echo "$line\\"
    done
  done
} > "$sph_sed"
build smallpt_sph -f "$sph_sed"
build smallpt_sph_xs -f "$sph_sed" -e "$xs"
build smallpt_sph16 -f "$sph_sed" -e '447a\	if (depth + 1 >= 16) return hit.e;'
build smallpt_sph16_xs -f "$sph_sed" -e '447a\	if (depth + 1 >= 16) return hit.e;' -e "$xs"
echo "built $OUT/smallpt_{nee,cos,uni,q05,sph,sph16} $OUT/smallpt_{nee,cos,uni,q05,sph,sph16}_xs $OUT/smallpt_{nee,cos}_omp"
