/*
 * spt_oracle_cli.c — command-line front end of the CPU oracle (TEST INFRASTRUCTURE ONLY).
 *   spt_oracle compat  W H SPP SEED nee|cos OUT.ppm     fp64 restatement of the reference (P0)
 *   spt_oracle counter W H SPP SEED nee|cos OUT.ppm     counter-mode contract (fp32, Philox)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "../include/spt.h"

int spt_oracle_compat_render(const spt_prim*, int, int, int, int, unsigned, int, double*);
int spt_oracle_write_ppm_d(const char*, int, int, const double*);
int spt_oracle_write_ppm_f(const char*, int, int, const float*);
int spt_oracle_counter_render(const spt_prim*, int, const spt_camera*, const spt_params*,
                              const int32_t*, int, float*, uint64_t*, int);
int spt_oracle_scene_cornell(spt_prim*);
void spt_oracle_default_params(spt_params*);
void spt_oracle_camera_spt(spt_camera*, float);

int main(int argc, char** argv) {
  spt_prim prims[64];
  int32_t n = 0;
  int w, h, spp, nee;
  unsigned seed;
  if (argc < 8) {
    fprintf(stderr, "usage: %s compat|counter W H SPP SEED nee|cos OUT.ppm\n", argv[0]);
    return 2;
  }
  w = atoi(argv[2]); h = atoi(argv[3]); spp = atoi(argv[4]); seed = (unsigned)strtoul(argv[5], 0, 10);
  nee = strcmp(argv[6], "cos") != 0;
  n = spt_oracle_scene_cornell(prims);
  if (!strcmp(argv[1], "compat")) {
    double* c = (double*)malloc(sizeof(double) * 3 * (size_t)w * (size_t)h);
    spt_oracle_compat_render(prims, n, w, h, spp, seed, nee, c);
    return spt_oracle_write_ppm_d(argv[7], w, h, c);
  } else {
    spt_params p;
    spt_camera cam;
    float* c = (float*)malloc(sizeof(float) * 3 * (size_t)w * (size_t)h);
    int32_t* rows = (int32_t*)malloc(sizeof(int32_t) * (size_t)h);
    uint64_t st[8];
    int y;
    spt_oracle_default_params(&p);
    p.width = w; p.height = h; p.spp = spp; p.seed = seed; p.nee_prob = nee ? 1.0f : 0.0f;
    spt_oracle_camera_spt(&cam, (float)w / (float)h);
    for (y = 0; y < h; y++) rows[y] = y;
    spt_oracle_counter_render(prims, n, &cam, &p, rows, h, c, st, 0);
    fprintf(stderr, "samples %llu path_rays %llu shadow_rays %llu vertices %llu misses %llu\n",
            (unsigned long long)st[0], (unsigned long long)st[1], (unsigned long long)st[2],
            (unsigned long long)st[3], (unsigned long long)st[7]);
    return spt_oracle_write_ppm_f(argv[7], w, h, c);
  }
}
