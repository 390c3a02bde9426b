// Standalone replay driver (profiling aid): runs the engine's association
// replay over a stream dumped by tools/micro/dump_stream.py, no Python.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include "../../include/eao_accel.h"
int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "gpurun_out/stream.bin";
  const int reps = argc > 2 ? atoi(argv[2]) : 3;
  FILE* f = fopen(path, "rb");
  if (!f) return 2;
  int n; if (fread(&n, 4, 1, f) != 1) return 3;
  struct Fr { int h[3]; std::vector<float> T, pos, uv; std::vector<int> boxes, ids; std::vector<uint8_t> bad; };
  std::vector<Fr> fr(n);
  for (auto& x : fr) {
    if (fread(x.h, 4, 3, f) != 3) return 4;
    x.T.resize(16); x.boxes.resize(5 * x.h[0]); x.ids.resize(x.h[1]); x.pos.resize(3 * x.h[1]);
    x.uv.resize(2 * x.h[1]); x.bad.resize(x.h[1]);
    if (fread(x.T.data(), 4, 16, f) != 16) return 5;
    if (x.h[0] && fread(x.boxes.data(), 4, x.boxes.size(), f) != x.boxes.size()) return 5;
    if (x.h[1] && fread(x.ids.data(), 4, x.ids.size(), f) != x.ids.size()) return 5;
    if (x.h[1] && fread(x.pos.data(), 4, x.pos.size(), f) != x.pos.size()) return 5;
    if (x.h[1] && fread(x.uv.data(), 4, x.uv.size(), f) != x.uv.size()) return 5;
    if (x.h[1] && fread(x.bad.data(), 1, x.bad.size(), f) != x.bad.size()) return 5;
  }
  eao_assoc* a;
  if (eao_assoc_create(0, 1 << 16, &a)) { printf("assoc: %s\n", eao_last_error()); return 6; }
  const float K[4] = {535.4f, 539.2f, 320.1f, 247.6f};
  for (int r = 0; r < reps; r++) {
    eao_replay* rp;
    eao_replay_create(a, "EAO", 640, 480, K, &rp);
    auto t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < n; t++) {
      std::vector<int> out(4 * fr[t].h[0] + 4);
      int rc = eao_replay_frame(rp, t + 1, fr[t].T.data(), fr[t].h[0], fr[t].boxes.data(), fr[t].h[1], fr[t].ids.data(),
                                fr[t].pos.data(), fr[t].uv.data(), fr[t].bad.data(), out.data());
      if (rc < 0) { printf("frame %d: %s\n", t, eao_last_error()); return 7; }
      if (fr[t].h[2]) eao_replay_local_mapping(rp);
    }
    double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    double pr[24]; eao_replay_profile(rp, pr);
    printf("rep %d: %.1f ms (%.0f us/frame) frame %.0f lm %.0f | iforest %.0f %.0f | np %.0f %.0f | rects %.0f %.0f"
           " | sections(us/frame) pts %.0f stats %.0f gpu0 %.0f assoc %.0f | spec %.0f | flush cls %.0f end %.0f | kick %.0f launch %.0f | retire %.0f x %.0f us | scan %.0f pack+launch %.0f\n", r,
           dt * 1e3, dt * 1e6 / n, pr[0] / 1e3, pr[1] / 1e3, pr[2], pr[3] / 1e3, pr[4], pr[5] / 1e3, pr[6], pr[7] / 1e3,
           pr[12] / n, pr[13] / n, pr[14] / n, pr[15] / n, pr[9], pr[16] / n, pr[17] / n, pr[18] / n, pr[19] / n, pr[20], pr[21] / n, pr[22] / n, pr[23] / n);
    eao_replay_destroy(rp);
  }
  return 0;
}
