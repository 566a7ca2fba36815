/*
 * spt_flops.h — frozen algorithmic FLOP model for roofline reporting.
 *
 * Counted from the reference source (/root/reference/src/smallpt.cpp), FMA = 2, add/sub/mul/div/
 * sqrt/sin/cos = 1 each, compares/selects = 0. Redundant reference work (the re-intersections at
 * :469/:476 whose result only feeds path_length, the repeated d.norm() at :471-472/:479) is NOT
 * counted. The kernel counts the events; FLOP = sum(events x constants) below.
 */
#ifndef SPT_FLOPS_H_
#define SPT_FLOPS_H_

/* per pixel-sample: jitter u,v (:533-534, 7), get_ray (:276-279, 15), normalise (:50-52, 10),
 * accumulate r += L*(1/spp) (:536, 6) */
#define SPT_FLOP_SAMPLE 40
/* per primitive test per ray: Rectangle_*::intersect (:102-112): sub, div, 2x(mul+add) */
#define SPT_FLOP_RECT 6
/* Sphere::intersect (:229-239): op 3, b 5, det 9, sqrt 1, t 1 */
#define SPT_FLOP_SPHERE 19
/* per shaded vertex: hit point o+d*t (:375, 6) + normal orientation dot (:123, 5) */
#define SPT_FLOP_VERTEX 11
/* extra for a sphere vertex normal (x-p).norm() (:247): 3 + 10 */
#define SPT_FLOP_SPHERE_NORMAL 13
/* per continuing (non-terminal) vertex: combine e + f.mult(L)*PDF*BRDF (:479) */
#define SPT_FLOP_COMBINE 12
/* per cosine-weighted direction (random_scattering :340-347) */
#define SPT_FLOP_COSINE 65
/* per NEE event: light sample (:365-367, 9) + normalise (10); per NEE light hit additionally
 * PDF (:471, 8) + BRDF (:472, 6) */
#define SPT_FLOP_NEE 19
#define SPT_FLOP_NEE_HIT 14

#endif /* SPT_FLOPS_H_ */
