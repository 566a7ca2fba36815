// smallpt_main.cpp — the reference's main() (smallpt.cpp:502-557) on the MI355X:
//   smallpt_amd [W H SPP [SEED [OUT.ppm]]] [--cos] [--uniform] [--reference-leaks] [--q Q]
//               [--specular | --classic | --mirror-glass | --spheres32 [--max-depth D]]
//               [--device N | --devices N] [--p6 | --pfm]
//   --uniform: random_scattering from the commented-out uniform hemisphere code (:352-359)
//   --reference-leaks: leaked paths go on from the miss vertex as the reference's (:371-377)
//                      instead of ending at their first miss (SPT_FLAG_REFERENCE_LEAKS)
//   --q Q: the NEE-mix probability of :464 (`q < Q`; 1 = HEAD, 0 = --cos)
//   --specular: smallpt's mirror and glass balls (SPEC/REFR, :481-495) in the HEAD room
//   --classic: the classic smallpt sphere box of the shipped image*.ppm (pure path tracing)
//   --mirror-glass: that box with smallpt's mirror and glass balls (pure path tracing)
//   --spheres32: config 5's 32-sphere scene (room + light of :288-294 and 32 DIFF spheres)
//   --devices N: row tiles sharded over GPUs 0..N-1, one RCCL gather to GPU 0 (spt_render_multi)
//   --repeat N: render N times (spt_render keeps its device context between calls) and print
//               each call's wall time beside its kernel time (tools/dropin_e2e.py)
// Same scene, camera (:521), clamp/toInt and P3 output; the pixel loop is one spt_render() call.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <iostream>

#include "smallpt.hpp"

using namespace smallpt_amd;

int main(int argc, char* argv[]) {
  int pos[4] = {512, 512, 16, 1};  // :507-508 defaults, seed 1
  const char* out = "image.ppm";
  bool cosine = false, uniform = false, specular = false, classic = false, mirror_glass = false;
  bool spheres = false, ref_leaks = false;
  int device = 0, devices = 0, max_depth = 0, npos = 0, format = SPT_IMAGE_P3, repeat = 1;
  float q = -1.0f;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--cos")) cosine = true;
    else if (!std::strcmp(argv[i], "--uniform")) uniform = true;
    else if (!std::strcmp(argv[i], "--reference-leaks")) ref_leaks = true;
    else if (!std::strcmp(argv[i], "--specular")) specular = true;
    else if (!std::strcmp(argv[i], "--classic")) classic = true;
    else if (!std::strcmp(argv[i], "--mirror-glass")) mirror_glass = true;
    else if (!std::strcmp(argv[i], "--spheres32")) spheres = true;
    else if (!std::strcmp(argv[i], "--max-depth") && i + 1 < argc) max_depth = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--q") && i + 1 < argc) q = (float)std::atof(argv[++i]);
    else if (!std::strcmp(argv[i], "--device") && i + 1 < argc) device = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--devices") && i + 1 < argc) devices = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--repeat") && i + 1 < argc) repeat = std::max(1, std::atoi(argv[++i]));
    else if (!std::strcmp(argv[i], "--p6")) format = SPT_IMAGE_P6;
    else if (!std::strcmp(argv[i], "--pfm")) format = SPT_IMAGE_PFM;
    else if (npos < 4) pos[npos++] = std::atoi(argv[i]);
    else out = argv[i];
  }
  const auto t1 = std::chrono::high_resolution_clock::now();
  spt_params p;
  spt_default_params(&p);
  p.width = pos[0]; p.height = pos[1]; p.spp = pos[2]; p.seed = (uint32_t)pos[3];
  const bool box = classic || mirror_glass;
  p.nee_prob = q >= 0.0f ? q : (cosine || box ? 0.0f : 1.0f);  // :464 (the sphere box: emission only)
  p.max_depth = max_depth;
  if (uniform) p.flags |= SPT_FLAG_UNIFORM_SCATTER;
  if (ref_leaks) p.flags |= SPT_FLAG_REFERENCE_LEAKS;
  p.device = device;
  Camera cam(LOOKFROM, Vec(50, 40, 5), Vec(0, 1, 0), 65, float(p.width) / float(p.height));  // :521
  spt_stats st{};
  std::vector<float> c;
  try {
    const std::vector<spt_prim> scene = classic ? smallpt_classic_scene()
                                        : mirror_glass ? smallpt_mirror_glass_scene()
                                        : specular ? cornell_specular_scene()
                                        : spheres ? spheres32_scene()
                                                  : cornell_scene();
    for (int k = 0; k < repeat; ++k) {
      const auto c0 = std::chrono::high_resolution_clock::now();
      if (devices > 0) {
        std::vector<int32_t> devs(devices);
        for (int j = 0; j < devices; ++j) devs[j] = j;
        c = render_multi(scene, cam, p, devs, &st);
      } else {
        c = render(scene, cam, p, &st);
      }
      const auto c1 = std::chrono::high_resolution_clock::now();
      if (repeat > 1)
        std::cout << "CALL " << k << " : WALL_MS " << std::chrono::duration<double, std::milli>(c1 - c0).count()
                  << "  KERNEL_MS " << st.kernel_ms << std::endl;
    }
  } catch (const std::exception& e) {
    std::cerr << "render failed: " << e.what() << std::endl;
    return 1;
  }
  const auto w0 = std::chrono::high_resolution_clock::now();
  if (write_ppm(out, p.width, p.height, c.data(), device, format)) {
    std::cerr << "cannot write " << out << ": " << spt_last_error() << std::endl;
    return 1;
  }
  const auto t2 = std::chrono::high_resolution_clock::now();
  std::cout << "WRITE_MS : " << std::chrono::duration<double, std::milli>(t2 - w0).count() << std::endl;
  const double samples = (double)p.width * p.height * p.spp;
  std::cout << "KERNEL_MS : " << st.kernel_ms << "  MSAMPLES/S : " << samples / (st.kernel_ms * 1e3)
            << "  VERTICES/SAMPLE : " << (double)st.vertices / samples << std::endl;
  std::cout << " DURATION : " << std::chrono::duration_cast<std::chrono::milliseconds>(t2 - t1).count()
            << std::endl;  // :554-556
  return 0;
}
