// gprof driver of the replay's host orchestration (development aid): the packed stream dumped by
// dump.py through eao_replay_run on the host-only harness (tests/native), `passes` times.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../../include/eao_accel.h"

extern "C" eao_assoc* harness_assoc_create();
template <class T>
static std::vector<T> rd(FILE* f, size_t n) {
  std::vector<T> v(n);
  if (n && fread(v.data(), sizeof(T), n, f) != n) exit(3);
  return v;
}
int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  const int passes = argc > 2 ? atoi(argv[2]) : 1;
  auto hdr = rd<int>(f, 4);
  const int n = hdr[0], nb = hdr[1], np = hdr[2];
  auto ids = rd<int>(f, n);
  auto T = rd<float>(f, 16 * (size_t)n);
  auto nbv = rd<int>(f, n);
  auto boxes = rd<int>(f, 5 * (size_t)nb);
  auto npt = rd<int>(f, n);
  auto mp = rd<int>(f, np);
  auto pos = rd<float>(f, 3 * (size_t)np);
  auto uv = rd<float>(f, 2 * (size_t)np);
  auto bad = rd<unsigned char>(f, np);
  auto kf = rd<unsigned char>(f, n);
  auto nl = rd<int>(f, n);
  size_t tl = 0;
  for (int x : nl) tl += x;
  auto lines = rd<float>(f, 4 * tl);
  fclose(f);
  const float K4[4] = {535.4f, 539.2f, 320.1f, 247.6f};
  std::vector<int> det(4 * (size_t)nb);
  for (int p = 0; p < passes; p++) {
    eao_assoc* a = harness_assoc_create();
    eao_replay* r = nullptr;
    if (eao_replay_create(a, hdr[3] ? "Full" : "EAO", 640, 480, K4, &r)) return 4;
    if (eao_replay_lines(r, n, nl.data(), lines.data())) return 5;
    const int rc = eao_replay_run(r, n, ids.data(), T.data(), nbv.data(), boxes.data(), npt.data(), mp.data(),
                                  pos.data(), uv.data(), bad.data(), kf.data(), det.data());
    printf("pass %d: rc %d\n", p, rc);
    eao_replay_destroy(r);
  }
  return 0;
}
