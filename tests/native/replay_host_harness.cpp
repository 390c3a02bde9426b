// CPU harness for the engine's host-side association orchestration
// (eao-slam_amd/csrc/replay.cpp): the three GPU primitives are served by the
// oracle so the decision logic can be debugged without a device. Test
// infrastructure only -- never part of the product.
#include <cstring>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include "../../eao-slam_amd/csrc/assoc.h"
#include "../../eao-slam_amd/csrc/shard.h"
#include "../../oracle/oracle.h"
#include <string>
#include <vector>

namespace eao {
static std::string g_err;
void set_error(const std::string& s) { g_err = s; }
CamDev make_cam(const eao_camera& c) {
  CamDev d;
  d.fx = c.fx; d.fy = c.fy; d.cx = c.cx; d.cy = c.cy;
  d.minX = 0; d.maxX = (float)c.img_w; d.minY = 0; d.maxY = (float)c.img_h;
  d.invW = 64.0f / d.maxX; d.invH = 48.0f / d.maxY;
  return d;
}
static bool g_in_rects_np = false;  // EAO_HARNESS_DUMP: tags the frame-start pairs
int AssocEngine::np_batch(int npairs, const float* fp, const uint8_t* fv, const int* foff, const int* flen,
                          const float* op, const uint8_t* ov, const int* ooff, const int* olen,
                          eao_np_stats* out, const Lane&, int, const double* const* os_ptr, const float* oth) {
  static FILE* dump = std::getenv("EAO_HARNESS_DUMP") ? std::fopen(std::getenv("EAO_HARNESS_DUMP"), "w") : nullptr;
  for (int p = 0; p < npairs; p++) {
    if (dump) {  // kind (fs: frame start, np: speculative / relaunch), pairs, m, n, valid m, kept valid n, kept n
      int mv = 0, nv = 0, nk = 0;
      for (int i = 0; i < flen[p]; i++) mv += fv[foff[p] + i] != 0;
      for (int i = 0; i < olen[p]; i++) {
        const bool k = !(os_ptr && os_ptr[p] && os_ptr[p][i] > (double)oth[p]);
        nk += k;
        nv += k && ov[ooff[p] + i];
      }
      std::fprintf(dump, "%s %d %d %d %d %d %d\n", g_in_rects_np ? "fs" : "np", npairs, flen[p], olen[p], mv, nv, nk);
    }
    std::vector<float> pts;
    std::vector<uint8_t> val;
    const double* os = os_ptr ? os_ptr[p] : nullptr;
    for (int i = 0; i < olen[p]; i++) {  // the forest's erasure, as the kernel applies it
      if (os && os[i] > (double)oth[p]) continue;
      pts.insert(pts.end(), op + 3 * (ooff[p] + i), op + 3 * (ooff[p] + i) + 3);
      val.push_back(ov[ooff[p] + i]);
    }
    orc_np_stats s;
    orc_np_test(flen[p], fp + 3 * foff[p], fv + foff[p], (int)val.size(), pts.data(), val.data(), &s);
    static_assert(sizeof(s) == sizeof(eao_np_stats), "layout");
    std::memcpy(&out[p], &s, sizeof(s));
  }
  return 0;
}
int AssocEngine::iforest_batch(int nclouds, const float* pts, const int* off, const int* len, uint32_t trees,
                               uint32_t seed, const uint32_t* sample, double* scores, const Lane&, int, int,
                               int, double*, double* scores2, const int* pk, const float* pth, unsigned char* pdst) {
  // fault injection (tests): EAO_HARNESS_FAIL_IFOREST=N fails the N-th forest launch (1-based)
  static int calls = 0;
  static const int fail_at = std::getenv("EAO_HARNESS_FAIL_IFOREST") ? std::atoi(std::getenv("EAO_HARNESS_FAIL_IFOREST")) : 0;
  if (++calls == fail_at) {
    set_error("harness: injected forest launch failure");
    return EAO_E_HIP;
  }
  static FILE* dump = std::getenv("EAO_HARNESS_DUMP") ? std::fopen((std::string(std::getenv("EAO_HARNESS_DUMP")) + ".if").c_str(), "w") : nullptr;
  for (int c = 0; c < nclouds; c++) {
    if (dump) std::fprintf(dump, "if %d %d\n", nclouds, len[c]);
    if (orc_iforest_scores(pts + 3 * off[c], len[c], trees, seed, sample[c], scores + off[c]))
      for (int i = 0; i < len[c]; i++) scores[off[c] + i] = NAN;  // Build() failed: nothing erased
    if (scores2)
      for (int i = 0; i < len[c]; i++) scores2[off[c] + i] = scores[off[c] + i];
    if (pdst)  // k_iforest_sum's outlier bit mask of the device-form exchange
      for (int j = 0; j < (len[c] + 7) / 8; j++) {
        unsigned v = 0;
        for (int b = 0; b < 8 && 8 * j + b < len[c]; b++)
          if (scores[off[c] + 8 * j + b] > (double)pth[c]) v |= 1u << b;
        pdst[pk[3 * c + 2] + j] = (unsigned char)v;
      }
  }
  return 0;
}
int AssocEngine::rects(const CamDev& cam, const float* T, int nclouds, const float* pts, const int* off,
                       const int* len, int* rect, uint8_t* ok, hipStream_t, const double* const* os_ptr,
                       const float* oth) {
  orc_camera c{(int)cam.maxX, (int)cam.maxY, cam.fx, cam.fy, cam.cx, cam.cy};
  for (int k = 0; k < nclouds; k++) {
    std::vector<float> kept;
    const double* os = os_ptr ? os_ptr[k] : nullptr;
    for (int i = 0; i < len[k]; i++)  // a pending forest's erasure, as the kernel applies it
      if (!(os && os[i] > (double)oth[k])) kept.insert(kept.end(), pts + 3 * (off[k] + i), pts + 3 * (off[k] + i) + 3);
    ok[k] = orc_project_rect(&c, T, (int)kept.size() / 3, kept.data(), rect + 4 * k) == 0;
  }
  return 0;
}
int AssocEngine::rects_np(const CamDev& cam, const float* T, int nclouds, const float* rpts, const int* roff,
                          const int* rlen, int* rect, uint8_t* ok, const double* const* ros, const float* rth,
                          int npairs, const float* fp, const uint8_t* fv, const int* foff, const int* flen,
                          const float* op, const uint8_t* ov, const int* ooff, const int* olen, eao_np_stats* out,
                          const Lane& s, int max_olen, const double* const* os_ptr, const float* oth) {
  rects(cam, T, nclouds, rpts, roff, rlen, rect, ok, s.s, ros, rth);
  g_in_rects_np = true;
  const int rc = np_batch(npairs, fp, fv, foff, flen, op, ov, ooff, olen, out, s, max_olen, os_ptr, oth);
  g_in_rects_np = false;
  return rc;
}
bool AssocEngine::iforest_fits(int max_len, int) const { return max_len <= IF_MAXN; }
int AssocEngine::stage_in(void* dst, const void* src, size_t bytes, const Lane&) {
  std::memcpy(dst, src, bytes);  // host "device" memory
  return EAO_OK;
}
AssocEngine::~AssocEngine() {}
}  // namespace eao

struct eao_assoc { eao::AssocEngine e; };
extern "C" const char* eao_last_error(void) { return eao::g_err.c_str(); }
namespace eao { AssocEngine* assoc_engine(eao_assoc* a) { return &a->e; } }
extern "C" eao_assoc* harness_assoc_create() { auto* a = new eao_assoc(); a->e.dev = 0; return a; }
// The RCCL exchanger is product-only. In its place eao_replay_shard_rccl gets a
// device-form exchanger over the all-gather callback set by harness_set_device_exchange
// (gloo from Python): "device" memory is host memory here, so the replay's device-form
// code paths (records written by iforest_batch / np_batch / rects_np into device buffers,
// gathered from there) run on the CPU against the oracle.
namespace eao {
namespace {
eao_allgather_fn g_dev_fn = nullptr;
void* g_dev_ctx = nullptr;
struct DeviceLoopExchanger : Exchanger {
  int world;
  std::vector<unsigned char> recv;
  explicit DeviceLoopExchanger(int w) : world(w) {}
  int allgather(const void*, void*, size_t) override {
    set_error("harness device exchanger: host form called");
    return EAO_E_ARG;
  }
  bool device_form() const override { return true; }
  // started exchanges gather at once (the callback is synchronous), in start order on every rank;
  // the ticket's records wait in their own buffer
  std::vector<std::vector<unsigned char>> tickets;
  std::vector<bool> busy;
  int start_device(const void* d_send, const ExReady&, size_t bytes, int* ticket) override {
    int k = 0;
    while (k < (int)busy.size() && busy[k]) k++;
    if (k == (int)busy.size()) {
      busy.push_back(false);
      tickets.emplace_back();
    }
    std::vector<unsigned char>& r = tickets[k];
    r.assign(bytes * world, 0xcd);
    if (world == 1) {
      std::memcpy(r.data(), d_send, bytes);
    } else if (!g_dev_fn || g_dev_fn(g_dev_ctx, d_send, r.data(), bytes)) {
      set_error("harness device exchanger: all-gather failed");
      return EAO_E_ARG;
    }
    busy[k] = true;
    *ticket = k;
    return EAO_OK;
  }
  int wait_device(int ticket, const unsigned char** out) override {
    if (ticket < 0 || ticket >= (int)busy.size() || !busy[ticket]) {
      set_error("harness device exchanger: unknown ticket");
      return EAO_E_STATE;
    }
    busy[ticket] = false;
    recv = tickets[ticket];
    *out = recv.data();
    return EAO_OK;
  }
};
}  // namespace
Exchanger* make_rccl_exchanger(int, int, int world, const void*, int* rc) {
  *rc = 0;
  return new DeviceLoopExchanger(world);
}
int AssocEngine::publish(const Lane&, void*, size_t, uint64_t*, uint64_t) {
  set_error("harness: no HSA lanes");  // the harness's lanes are HIP-stream lanes (never called)
  return EAO_E_STATE;
}
}  // namespace eao
extern "C" void harness_set_device_exchange(eao_allgather_fn fn, void* ctx) {
  eao::g_dev_fn = fn;
  eao::g_dev_ctx = ctx;
}
extern "C" void harness_set_events_never(int v) { fake_events_never() = v; }

// launch lanes (hsa_lane.h): HIP-stream lanes only; completion markers follow the fake events
namespace eao {
bool hsa_lanes_available(int) { return false; }
int lanes_open(Lane* l, int n, bool, int) {
  for (int i = 0; i < n; i++) l[i] = Lane((hipStream_t)1);
  return 0;
}
void lane_close(Lane& l) { l = Lane(); }
int lane_sync(const Lane&) { return 0; }
void done_close(Done& d) { d = Done(); }
int lane_record(const Lane&, Done& d) {
  d.e = (hipEvent_t)1;
  return 0;
}
int lane_wait(const Lane&, const Done&) { return 0; }
hipError_t done_query(const Done& d) { return d.e ? hipEventQuery(d.e) : hipSuccess; }
void* bar_alloc(int, size_t) { return nullptr; }
void bar_free(void*) {}
void lane_bar_written(const Lane&, const void*) {}
}  // namespace eao
