// baseline_mt.cpp -- the all-cores leg of bench.py's CPU baseline (TEST INFRASTRUCTURE ONLY).
//
// BASELINE.md §2 / SURVEY.md §8d: besides the reference's own single Tracking
// thread, time the restatement frame-parallel over the host's cores. Frames are
// independent units for ORBextractor::operator() (src/ORBextractor.cc:1043-1105),
// and the motion-model search of frame t (SearchByProjection(Cur, Last, 15, mono),
// src/ORBmatcher.cc:1328-1470) needs only frames t-1 and t, so both phases are
// spread over `threads` std::threads, each taking every threads-th unit. The
// association stays sequential (it is one decision chain) and is timed by the
// caller on one thread.
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "oracle.h"

extern "C" {

// frames [n][h][w] u8; outputs per frame slot of `cap`: kps, desc (cap x 32), nkp.
// Matching of pair (t-1, t) for t >= 1 uses frame t-1's keypoints and descriptors with
// the map state has[(t-1) cap], mpos[(t-1) cap][3] and Tcw[t] (16 floats), writing
// match[t cap] and nmatch[t]. Returns the wall time of the two phases in seconds.
double orc_extract_match_mt(const uint8_t* frames, int n, int w, int h, int nfeatures, float scale_factor,
                            int nlevels, int iniTh, int minTh, const orc_camera* cam, const float* Tcw,
                            const uint8_t* has, const float* mpos, float th, int check_ori, const float* scales,
                            int cap, int threads, orc_keypoint* kps, uint8_t* desc, int* nkp, int32_t* match,
                            int* nmatch) {
  if (threads < 1) threads = 1;
  const auto t0 = std::chrono::steady_clock::now();
  std::atomic<int> next{0};
  auto extract = [&]() {
    for (int t; (t = next.fetch_add(1)) < n;)
      orc_orb_extract(frames + (size_t)t * w * h, w, h, nfeatures, scale_factor, nlevels, iniTh, minTh,
                      kps + (size_t)t * cap, desc + (size_t)t * cap * 32, cap, &nkp[t]);
  };
  std::vector<std::thread> pool;
  for (int k = 0; k < threads; k++) pool.emplace_back(extract);
  for (auto& th_ : pool) th_.join();
  pool.clear();
  next = 1;
  nmatch[0] = 0;
  auto matchp = [&]() {
    for (int t; (t = next.fetch_add(1)) < n;)
      nmatch[t] = orc_search_by_projection_motion(
          cam, Tcw + 16 * (size_t)t, th, check_ori, nkp[t - 1], kps + (size_t)(t - 1) * cap,
          has + (size_t)(t - 1) * cap, mpos + (size_t)(t - 1) * cap * 3, desc + (size_t)(t - 1) * cap * 32, nkp[t],
          kps + (size_t)t * cap, desc + (size_t)t * cap * 32, nlevels, scales, match + (size_t)t * cap);
  };
  for (int k = 0; k < threads; k++) pool.emplace_back(matchp);
  for (auto& th_ : pool) th_.join();
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

}  // extern "C"
