// The drop-in per-callback path from C++ straight on the C-ABI (what a ROS node linking
// libc3hlac_mi355x.so sees, detect_object.cpp:139-186): host cloud -> c3h_voxelize ->
// c3h_extract -> c3h_search -> host lists, one frame at a time; no Python in the loop.
// Input: a file written by bench.py (write_native_frames) (scenes + the search bases).
// Build: make -C mapping-private_amd (target lib/single_frame_native, rpath to the library)
// Usage: mapping-private_amd/lib/single_frame_native DATA FRAMES [LISTS]  -> one JSON line (medians, ms per
// frame); LISTS: the detection lists (M c3h_det per scene, rank 1) of the first timed frame of each scene
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "c3hlac_mi355x.h"

static bool read_all(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n; }

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s DATA FRAMES\n", argv[0]);
    return 1;
  }
  const int frames = atoi(argv[2]);
  FILE* f = fopen(argv[1], "rb");
  if (!f) {
    fprintf(stderr, "cannot open %s\n", argv[1]);
    return 1;
  }
  int32_t hdr[8];
  if (!read_all(f, hdr, sizeof(hdr))) return 1;
  const int ns = hdr[0], D = hdr[1], F = hdr[2], M = hdr[3], r = hdr[4], variant = hdr[5], subdiv = hdr[6];
  float fh[2];  // leaf, exist threshold
  if (!read_all(f, fh, sizeof(fh))) return 1;
  int32_t thr[3], box[3];
  if (!read_all(f, thr, sizeof(thr)) || !read_all(f, box, sizeof(box))) return 1;
  std::vector<float> axis((size_t)D * F), var(D), q((size_t)M * r * D);
  if (!read_all(f, axis.data(), axis.size() * 4) || !read_all(f, var.data(), var.size() * 4) ||
      !read_all(f, q.data(), q.size() * 4))
    return 1;
  std::vector<std::vector<float>> scenes(ns);
  for (auto& s : scenes) {
    int64_t n;
    if (!read_all(f, &n, 8)) return 1;
    s.resize((size_t)n * 4);
    if (!read_all(f, s.data(), s.size() * 4)) return 1;
  }
  fclose(f);
  c3h_ctx* ctx = nullptr;
  if (c3h_create(0, &ctx) != C3H_OK) {
    fprintf(stderr, "c3h_create failed\n");
    return 1;
  }
  int rc = c3h_search_setup(ctx, axis.data(), var.data(), D, F, q.data(), M, r, nullptr, 0);
  if (rc == C3H_OK) rc = c3h_set_rank(ctx, 1);
  if (rc != C3H_OK) {
    fprintf(stderr, "setup: %s\n", c3h_last_error(ctx));
    return 1;
  }
  c3h_extract_params p{};
  p.variant = variant;
  for (int a = 0; a < 3; ++a) p.thr[a] = thr[a];
  p.subdiv = subdiv;
  p.color_mode = C3H_COLOR_C3_DOUBLE;
  std::vector<c3h_det> out((size_t)M), keep((size_t)M * ns);
  std::vector<double> e2e, ph[3];
  int found = 0;
  auto frame = [&](int i, bool record) -> int {
    const auto& s = scenes[i % ns];
    c3h_grid_info gi;
    int32_t sb[3];
    int64_t hn;
    const auto t0 = std::chrono::steady_clock::now();
    int e = c3h_voxelize(ctx, s.data(), (int64_t)(s.size() / 4), 0, fh[0], INFINITY, &gi);
    const auto t1 = std::chrono::steady_clock::now();
    if (e == C3H_OK) e = c3h_clean_max(ctx);  // search_obj.cleanData() (detect_object.cpp:169)
    if (e == C3H_OK) e = c3h_extract(ctx, &p, sb, &hn);
    const auto t2 = std::chrono::steady_clock::now();
    if (e == C3H_OK) e = c3h_search(ctx, box, (int32_t)fh[1], 1, 0, out.data());
    const auto t3 = std::chrono::steady_clock::now();
    if (e < 0) return e;
    if (record) {
      const auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
      e2e.push_back(ms(t0, t3));
      ph[0].push_back(ms(t0, t1));
      ph[1].push_back(ms(t1, t2));
      ph[2].push_back(ms(t2, t3));
      found += out[0].score > 0 ? 1 : 0;
      if (i < ns) std::copy(out.begin(), out.end(), keep.begin() + (size_t)i * M);
    }
    return C3H_OK;
  };
  for (int i = 0; i < 2 * ns; ++i)  // untimed: buffers sized for the scenes
    if (frame(i, false) != C3H_OK) {
      fprintf(stderr, "frame: %s\n", c3h_last_error(ctx));
      return 1;
    }
  for (int i = 0; i < frames; ++i)
    if (frame(i, true) != C3H_OK) {
      fprintf(stderr, "frame: %s\n", c3h_last_error(ctx));
      return 1;
    }
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
  };
  printf("{\"frames\": %d, \"ms_per_frame_end_to_end\": %.4f, \"phases_ms_per_frame\": {\"voxelize\": %.4f, "
         "\"c3hlac\": %.4f, \"search\": %.4f}, \"frames_with_detection\": %d}\n",
         frames, med(e2e), med(ph[0]), med(ph[1]), med(ph[2]), found);
  c3h_destroy(ctx);
  if (argc > 3) {
    FILE* o = fopen(argv[3], "wb");
    if (!o || fwrite(keep.data(), sizeof(c3h_det), keep.size(), o) != keep.size()) {
      fprintf(stderr, "cannot write %s\n", argv[3]);
      return 1;
    }
    fclose(o);
  }
  return 0;
}
