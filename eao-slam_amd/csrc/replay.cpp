// replay.cpp -- the EAO association pass on the engine (host orchestration).
//
// Mirrors the object section of Tracking::TrackWithMotionModel
// (reference src/Tracking.cc:1241-1696), Object_2D::ObjectDataAssociation /
// Object_Map::DataAssociateUpdate (src/Object.cc:162-710, 1313-1554) and the
// LocalMapping object maintenance (src/LocalMapping.cc:772-882) as a
// deterministic single-threaded replay.
//
// Work split (DESIGN.md "Association"):
//   GPU  NoParaDataAssociation rank statistics for every (detection, object)
//        pair of a frame in ONE launch (k_np_pairs), re-issued only for a
//        class whose objects an earlier detection of the frame changed;
//        isolation forests of every object updated in the frame in ONE launch
//        (k_iforest_build/score), deferred until the object's points are next
//        read (exact: only same-class detections or end-of-frame read them);
//        projected rects of all recent objects in ONE launch (k_rects).
//   host the sequential decision logic (first-wins order is part of the
//        semantics), O(n) bookkeeping, and the duplicate-point test as an
//        O(m+n) exact-bit-pattern hash instead of the reference's O(m*n) scan.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <array>
#include <chrono>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/eao_accel.h"
#include "assoc.h"
#include "common.h"
#include "shard.h"


// Host-side waits of the association chain spin on hipEventQuery: a blocking
// hipEventSynchronize / hipStreamSynchronize may park the thread and pay a
// wake-up per wait, and the chain waits a few times per frame.
static const bool g_spin_wait = [] {
  const char* v = getenv("EAO_BLOCKING_WAIT");  // A/B switch for measurements
  return !(v && v[0] == '1');
}();
// A/B switch for measurements: EAO_NO_LOOKAHEAD=1 disables the look-ahead of eao_replay_run
static const bool g_lookahead = [] {
  const char* v = getenv("EAO_NO_LOOKAHEAD");
  return !(v && v[0] == '1');
}();
// Outputs written straight into pinned host memory (frame-start stats / rects, forest scores,
// speculative NP stats) are pre-filled with patterns no kernel writes (a NaN payload the
// hardware never produces; a byte no flag takes), and the host waits until every word it needs
// has been overwritten -- or until the launch's event completes, whichever comes first: the
// data lands a few microseconds before the command processor's end-of-kernel signal.
// EAO_SENTINEL_WAIT=0 waits on the events only (A/B switch).
static hipError_t spin_event_plain(const eao::Done& e) {
  for (;;) {
    const hipError_t r = eao::done_query(e);
    if (r != hipErrorNotReady) return r;
    __builtin_ia32_pause();
  }
}
// look-ahead steps 1-2 run over kPrepChunk points per step, so a wait the look-ahead fills
// notices its GPU result within one short step (EAO_PREP_CHUNK: A/B switch)
static const int kPrepChunk = [] {
  const char* v = getenv("EAO_PREP_CHUNK");
  const int c = v ? atoi(v) : 0;
  return c > 0 ? c : 128;
}();
// test switch: EAO_LOOKAHEAD_EAGER=1 runs a wait's look-ahead to completion whatever the wait's
// state (the CPU harness's kernels finish at launch, so its waits would otherwise never fill)
static const bool g_la_eager = [] {
  const char* v = getenv("EAO_LOOKAHEAD_EAGER");
  return v && v[0] == '1';
}();
// HSA lanes: a forest batch's packed inputs written straight into device memory through the BAR
// instead of pinned memory + k_stage (EAO_BAR_INPUTS=0: A/B switch)
static const bool g_bar_inputs = [] {
  const char* v = getenv("EAO_BAR_INPUTS");
  return !(v && v[0] == '0');
}();
// ... and the frame start's (EAO_BAR_FS=0: A/B switch)
static const bool g_bar_fs = [] {
  const char* v = getenv("EAO_BAR_FS");
  return g_bar_inputs && !(v && v[0] == '0');
}();
// sharded exchanges started where their result is read (EAO_SHARD_EAGER=1: with their launches --
// no gain measured, and one stream's waits then queue in launch order, not in the order of need:
// profiles/r06_ab_shard_eager.txt)
static const bool g_shard_eager = [] {
  const char* v = getenv("EAO_SHARD_EAGER");
  return v && v[0] == '1';
}();
// ComputeMeanAndStandard skipped when its inputs repeat its last call's (EAO_MS_MEMO=0: always
// computed, A/B and check)
static const bool g_ms_memo = [] {
  const char* v = getenv("EAO_MS_MEMO");
  return !(v && v[0] == '0');
}();
// EAO_MS_VERIFY=1: every skip also checks each held point against the object's change mark
static const bool g_ms_verify = [] {
  const char* v = getenv("EAO_MS_VERIFY");
  return v && v[0] == '1';
}();
// sharded replays on the HSA lanes (EAO_SHARD_HSA=0: HIP streams, A/B switch)
static const bool g_shard_hsa = [] {
  const char* v = getenv("EAO_SHARD_HSA");
  return !(v && v[0] == '0');
}();
static const bool g_sentinel = [] {
  const char* v = getenv("EAO_SENTINEL_WAIT");
  return !(v && v[0] == '0');
}();
static constexpr uint32_t kSent32 = 0x7FBADBADu;          // int / float words
static constexpr uint64_t kSent64 = 0x7FF4DEADBEEFCAFEull;  // double words
static constexpr uint8_t kSent8 = 0xAB;                    // flag bytes
static inline uint32_t ld32(const void* p) { return __atomic_load_n((const uint32_t*)p, __ATOMIC_RELAXED); }
static inline uint64_t ld64(const void* p) { return __atomic_load_n((const uint64_t*)p, __ATOMIC_RELAXED); }
static inline uint8_t ld8(const void* p) { return __atomic_load_n((const uint8_t*)p, __ATOMIC_RELAXED); }
static void fill32(void* p, size_t words) {
  uint32_t* q = (uint32_t*)p;
  for (size_t i = 0; i < words; i++) q[i] = kSent32;
}
static void fill64(void* p, size_t words) {
  uint64_t* q = (uint64_t*)p;
  for (size_t i = 0; i < words; i++) q[i] = kSent64;
}
// wait for `ready()` (sentinels overwritten) or the event, whichever comes first.
// Returning on the outputs alone is safe because the kernels that write these pinned outputs
// (k_rects_np / k_np_pairs via np_pair_body and rects_body, k_iforest_sum) keep three rules:
//   1. every output word the host waits for is stored exactly once, with its final value;
//   2. a workgroup's output stores follow all of its reads of the pinned inputs (and k_stage,
//      which copies a forest batch's pinned inputs to the device, precedes the tree kernel in
//      stream order), so a buffer is free for refilling once every output has landed;
//   3. no output word can equal its fill pattern (kSent32 / kSent64 are NaN payloads the
//      hardware never produces; kSent8 is no flag value).
// A fault after the outputs have landed is reported when the launch's event is queried before
// its buffers are reused (rects_np_launch, kick).
// (the wait's completion marker is a HIP event or an HSA signal, hsa_lane.h; a blocking wait
// applies to events only)
template <class Ready>
static hipError_t spin_ready(const eao::Done& e, Ready&& ready) {
  if (!g_sentinel || !g_spin_wait) return g_spin_wait || !e.e ? spin_event_plain(e) : hipEventSynchronize(e.e);
  for (;;) {
    if (ready()) return hipSuccess;
    const hipError_t r = eao::done_query(e);
    if (r != hipErrorNotReady) return r;
    __builtin_ia32_pause();
  }
}
static hipError_t spin_event(const eao::Done& e) {
  if (!g_spin_wait && e.e) return hipEventSynchronize(e.e);
  for (;;) {
    const hipError_t r = eao::done_query(e);
    if (r != hipErrorNotReady) return r;
    __builtin_ia32_pause();
  }
}

namespace eao {

static const float kTTable[122][9] = {
#include "t_table.inc"
};

namespace {

struct IRect {
  int x = 0, y = 0, w = 0, h = 0;
  IRect() {}
  IRect(int a, int b, int c, int d) : x(a), y(b), w(c), h(d) {}
  int area() const { return w * h; }
  bool contains_f(float u, float v) const {  // Rect::contains(Point(cvRound(u), cvRound(v)))
    return contains_i((int)lrintf(u), (int)lrintf(v));
  }
  bool contains_i(int px, int py) const { return x <= px && px < x + w && y <= py && py < y + h; }
};
inline IRect rect_trunc(float x, float y, float w, float h) { return IRect((int)x, (int)y, (int)w, (int)h); }
inline IRect rect_and(const IRect& a, const IRect& b) {
  const int x1 = std::max(a.x, b.x), y1 = std::max(a.y, b.y);
  const int w = std::min(a.x + a.w, b.x + b.w) - x1, h = std::min(a.y + a.h, b.y + b.h) - y1;
  return (w <= 0 || h <= 0) ? IRect() : IRect(x1, y1, w, h);
}
// Converter::bboxOverlapratio / Former / Latter, src/Converter.cc:194-212
inline float ov_iou(const IRect& a, const IRect& b) {
  const int o = rect_and(a, b).area();
  return (float)o / ((float)(a.area() + b.area() - o));
}
inline float ov_former(const IRect& a, const IRect& b) { return (float)rect_and(a, b).area() / ((float)a.area()); }
inline float ov_latter(const IRect& a, const IRect& b) { return (float)rect_and(a, b).area() / ((float)b.area()); }

struct Pose {
  float T[16];
  float fx, fy, cx, cy;
  int cols, rows;
  // Rcw*P + tcw (OpenCV small-gemm rounding) then the Object.cc projection
  void cam(const float* P, float* pc) const {
    for (int r = 0; r < 3; r++) {
      const float t = T[4 * r] * P[0] + T[4 * r + 1] * P[1] + T[4 * r + 2] * P[2];
      pc[r] = (float)((double)t + (double)T[4 * r + 3]);
    }
  }
  void proj(const float* P, float& u, float& v) const {
    float pc[3];
    cam(P, pc);
    const float iz = (float)(1.0 / pc[2]);
    u = fx * pc[0] * iz + cx;
    v = fy * pc[1] * iz + cy;
  }
};

struct MapPt {
  int id = 0;
  float pos[3] = {0, 0, 0};
  bool bad = false;
  float fu = 0, fv = 0;  // MapPoint::feature (current-frame keypoint)
  float pu = 0, pv = 0;  // projection under the current pose (cached per pose epoch)
  unsigned proj_epoch = 0;
  uint64_t ver = 0;  // the engine's point epoch at the last change of pos / bad
  // object_id_vector: a handful of (object id, count) entries per point,
  // only ever looked up (never iterated), so a flat vector suffices
  std::vector<std::pair<int, int>> votes;
  int* vote_of(int id) {
    for (auto& v : votes)
      if (v.first == id) return &v.second;
    return nullptr;
  }
  void vote_insert(int id, int c) {  // std::map::insert: no-op if present
    if (!vote_of(id)) votes.push_back({id, c});
  }
};

struct Obj;
struct Det {  // Object_2D
  int cls = -1;
  float score = 0;  // always 0
  int bx = 0, by = 0, bw = 0, bh = 0;
  IRect box, feat;
  std::vector<MapPt*> pts;
  float sum[3] = {0, 0, 0}, pos[3] = {0, 0, 0};
  bool bad = false;
  int mnId = -1, method = 0, index = -1;
  unsigned long fid = 0;  // the frame it was detected in
  Obj* alias = nullptr;  // _Pos shares mCenter3D's buffer (Object.cc:677, Tracking.cc:2563)
  // mObjLinesEigen (Tracking.cc:2524): the line angles SampleObjYaw reads, in degrees
  // as (double)(atan2f-rounded angle * 180) / pi -- only kept for yaw-sampled classes
  std::vector<double> line_deg;
  const float* P() const;
};

struct Obj {  // Object_Map
  std::vector<Det*> frames;
  IRect last, lastlast, proj;
  int id = 0, cls = 0, conf = 0, last_add = 0, lastlast_add = 0;
  std::vector<MapPt*> pts;
  float sum[3] = {0, 0, 0}, center[3] = {0, 0, 0}, sd[3] = {0, 0, 0}, csd[3] = {0, 0, 0};
  float csd_all = 0;
  std::map<int, int> reobj, same;
  bool bad = false;
  // cuboid (Cuboid3D)
  double corner[8][3], center_c[3] = {0, 0, 0};
  float xmn = 0, xmx = 0, ymn = 0, ymx = 0, zmn = 0, zmx = 0, lenth = 0, width = 0, height = 0;
  double q[4] = {1, 0, 0, 0}, t[3] = {0, 0, 0}, qn[4] = {1, 0, 0, 0}, tn[3] = {0, 0, 0};
  float rotY = 0, rotP = 0, rotR = 0, rmax = 0;
  double corner_w[8][3] = {};                  // corner_k_w (pose_without_yaw)
  std::vector<std::array<float, 5>> angles;    // mvAngleTimesAndScore
  float err_par = 0, err_yaw = 0;              // mfErrorParallel, mfErroeYaw
  bool yaw_due = false;                        // step 10.6 deferred behind the pending forest
  float yawT[16];                              // ... with the pose of its frame
  int pending = 0;  // 0 none, 1 iForest, 2 iForest then ComputeMeanAndStandard
  int slot = -1;    // in-flight isolation-forest slot, -1 if not launched
  // Effects of later detections of the same frame that depend on this object's pending
  // forest (it was updated earlier in the frame, so it can no longer be associated this
  // frame -- every such effect is a vote or a projected-rect recompute): applied in order
  // when the forest completes, with the pose of their frame (ReplayEngine::associate).
  // DFR_T: the t-test step of a later detection (Object.cc:497-620) whose rect overlap
  // with this object reads the post-forest projected rect; mode 0 a vote for the
  // detection's associated object, 1 (before the t-test winner, or no winner) a failed
  // update (rect recompute) if in vT else a vote, 2 (after the winner) a vote
  enum { DFR_PROJ = 0, DFR_PROJ_IF_NP = 1, DFR_VOTE_IF_NP = 2, DFR_T = 3 };
  struct Dfr {
    int kind;
    Det* det;     // the detection whose NP verdict against this object decides (kinds 1, 2)
    Obj* target;  // the object that receives the vote (kinds 2, 3)
    uint8_t mode = 0, t8 = 0, m10 = 0, m4 = 0;  // DFR_T: mode and the t-test outcomes
  };
  std::vector<Dfr> dfr;
  float dfrT[16];
  bool proj_dfr = false;  // a projected-rect recompute is among them
  // ComputeMeanAndStandard's inputs at its last call (ReplayEngine::mean_std): a call whose inputs
  // are all the same -- the point list, no point moved or turned bad since (the engine's epoch),
  // the frames' positions, the angles and the cuboid centre it starts from -- computes the same
  // outputs into the same state, and is skipped
  uint64_t ms_epoch = ~0ull;
  uint64_t pt_chg = 0;  // the point epoch of the last change of a point it may hold (one that voted for it)
  std::vector<MapPt*> ms_pts;
  std::vector<float> ms_fp;  // the frames' P(), 3 per frame
  float ms_rot[3] = {0, 0, 0};
  double ms_cc_in[3] = {0, 0, 0}, ms_cc_out[3] = {0, 0, 0};
  // the point list big_to_small left at its last call: none of them inside bts_box at epoch bts_epoch
  uint64_t bts_epoch = ~0ull;
  float bts_box[6] = {0, 0, 0, 0, 0, 0};
  std::vector<MapPt*> bts_pts;
  // the positions of ms_pts at that call (x block, y block, z block): valid while ms_epoch is
  std::vector<float> ms_pos;
};
const float* Det::P() const { return alias ? alias->center : pos; }

// Eigen 3.2 Quaternion(Matrix3d) + g2o SE3Quat::normalizeRotation
void quat_from_R(const double R[3][3], double q[4]) {
  double t = (R[0][0] + R[1][1]) + R[2][2];
  if (t > 0) {
    t = std::sqrt(t + 1.0);
    q[0] = 0.5 * t;
    t = 0.5 / t;
    q[1] = (R[2][1] - R[1][2]) * t;
    q[2] = (R[0][2] - R[2][0]) * t;
    q[3] = (R[1][0] - R[0][1]) * t;
  } else {
    int i = 0;
    if (R[1][1] > R[0][0]) i = 1;
    if (R[2][2] > R[i][i]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    t = std::sqrt(R[i][i] - R[j][j] - R[k][k] + 1.0);
    double c[3];
    c[i] = 0.5 * t;
    t = 0.5 / t;
    q[0] = (R[k][j] - R[j][k]) * t;
    c[j] = (R[j][i] + R[i][j]) * t;
    c[k] = (R[k][i] + R[i][k]) * t;
    q[1] = c[0];
    q[2] = c[1];
    q[3] = c[2];
  }
  if (q[0] < 0)
    for (int a = 0; a < 4; a++) q[a] = -q[a];
  const double nrm = std::sqrt(((q[1] * q[1] + q[3] * q[3]) + (q[2] * q[2] + q[0] * q[0])));
  for (int a = 0; a < 4; a++) q[a] = q[a] / nrm;
}
// Eigen's q * v: uv = 2 (q.vec x v); v + w uv + q.vec x uv. Scalars, not arrays: g++
// vectorises the array form into 16-byte reloads of 8-byte stores (store-forward stalls)
inline void qrot(const double q[4], const double v[3], double o[3]) {
  const double x = q[1], y = q[2], z = q[3], w = q[0];
  const double v0 = v[0], v1 = v[1], v2 = v[2];
  double u0 = y * v2 - z * v1, u1 = z * v0 - x * v2, u2 = x * v1 - y * v0;
  u0 += u0;
  u1 += u1;
  u2 += u2;
  const double c0 = y * u2 - z * u1, c1 = z * u0 - x * u2, c2 = x * u1 - y * u0;
  o[0] = v0 + w * u0 + c0;
  o[1] = v1 + w * u1 + c1;
  o[2] = v2 + w * u2 + c2;
}
inline void se3_apply(const double q[4], const double t[3], const double v[3], double o[3]) {
  double r[3];
  qrot(q, v, r);
  for (int a = 0; a < 3; a++) o[a] = r[a] + t[a];
}
// SE3Quat::inverse(): (conj(q), -(conj(q) * t))
void se3_inverse(const double q[4], const double t[3], double qc[4], double ti[3]) {
  qc[0] = q[0];
  qc[1] = -q[1];
  qc[2] = -q[2];
  qc[3] = -q[3];
  const double mt[3] = {t[0] * -1., t[1] * -1., t[2] * -1.};
  qrot(qc, mt, ti);
}
void se3_inv_apply(const double q[4], const double t[3], const double v[3], double o[3]) {
  double qc[4], ti[3];
  se3_inverse(q, t, qc, ti);
  se3_apply(qc, ti, v, o);
}

// exact-equality key for the duplicate test cv::countNonZero(a - b) == 0
// (Object.cc:1464-1477): equal iff every coordinate difference is 0, i.e.
// same value with -0 == +0; NaN/Inf never compare equal (Inf - Inf = NaN).
struct PosKey {
  uint32_t a, b, c;
  bool operator==(const PosKey& o) const { return a == o.a && b == o.b && c == o.c; }
};
struct PosHash {
  size_t operator()(const PosKey& k) const {
    uint64_t h = k.a * 0x9E3779B97F4A7C15ull;
    h ^= (k.b + 0x7F4A7C15ull) * 0xC2B2AE3D27D4EB4Full;
    h ^= (k.c + 0x165667B1ull) * 0x27D4EB2F165667C5ull;
    return (size_t)(h ^ (h >> 29));
  }
};
// open-addressing set of PosKeys, reused across calls (generation stamps
// instead of clearing)
struct PosSet {
  std::vector<PosKey> key;
  std::vector<uint32_t> gen;
  uint32_t cur = 0;
  size_t mask = 0;
  void reset(size_t n) {
    size_t cap = 64;
    while (cap < 2 * n + 16) cap <<= 1;
    if (cap > key.size()) {
      key.assign(cap, PosKey{0, 0, 0});
      gen.assign(cap, 0);
      cur = 0;
    }
    mask = key.size() - 1;
    if (++cur == 0) {
      std::fill(gen.begin(), gen.end(), 0);
      cur = 1;
    }
  }
  // returns true if k was inserted (absent before)
  bool insert(const PosKey& k) {
    size_t h = PosHash()(k) & mask;
    while (gen[h] == cur) {
      if (key[h] == k) return false;
      h = (h + 1) & mask;
    }
    gen[h] = cur;
    key[h] = k;
    return true;
  }
  bool contains(const PosKey& k) const {
    size_t h = PosHash()(k) & mask;
    while (gen[h] == cur) {
      if (key[h] == k) return true;
      h = (h + 1) & mask;
    }
    return false;
  }
};

bool pos_key(const float* p, PosKey& k) {
  uint32_t u[3];
  for (int i = 0; i < 3; i++) {
    if (!std::isfinite(p[i])) return false;
    const float v = p[i] == 0.0f ? 0.0f : p[i];
    std::memcpy(&u[i], &v, 4);
  }
  k = PosKey{u[0], u[1], u[2]};
  return true;
}

// min / max of v[0..n) exactly as the sequential std::min / std::max scan from (mn, mx) would
// leave them: eight independent lanes (the scan's select keeps NaNs out, as the scan does), and
// the sequential scan again when a result is zero (the one case where the lanes' tie order could
// pick the other sign of zero)
void minmax_scan(const float* v, size_t n, float& mn, float& mx) {
  float a[8], b[8];
  for (int k = 0; k < 8; k++) {
    a[k] = mn;
    b[k] = mx;
  }
  size_t i = 0;
  for (; i + 8 <= n; i += 8)
    for (int k = 0; k < 8; k++) {
      a[k] = v[i + k] < a[k] ? v[i + k] : a[k];
      b[k] = b[k] < v[i + k] ? v[i + k] : b[k];
    }
  float m0 = a[0], m1 = b[0];
  for (int k = 1; k < 8; k++) {
    m0 = a[k] < m0 ? a[k] : m0;
    m1 = m1 < b[k] ? b[k] : m1;
  }
  for (; i < n; i++) {
    m0 = v[i] < m0 ? v[i] : m0;
    m1 = m1 < v[i] ? v[i] : m1;
  }
  if (m0 == 0.0f || m1 == 0.0f) {
    float s0 = mn, s1 = mx;
    for (size_t j = 0; j < n; j++) {
      s0 = std::min(s0, v[j]);
      s1 = std::max(s1, v[j]);
    }
    m0 = s0;
    m1 = s1;
  }
  mn = m0;
  mx = m1;
}

// ComputeMeanAndStandard's cuboid pass: every position through the inverse object pose
// (Eigen's q * v + t in double), rounded to float. Gathered input, one point per iteration with no
// dependence between points: vectorised (AVX2 clone where the host has it), bit-identical per point
// (host code: the device compilation pass of this file sees no clones)
#if defined(__HIP_DEVICE_COMPILE__)
#define EAO_HOST_CLONES
#else
#define EAO_HOST_CLONES __attribute__((target_clones("avx2", "default")))
#endif
EAO_HOST_CLONES
void se3_batch(const double qi[4], const double ti[3], size_t n, const float* __restrict__ px,
               const float* __restrict__ py, const float* __restrict__ pz, float* __restrict__ ox,
               float* __restrict__ oy, float* __restrict__ oz) {
  const double x = qi[1], y = qi[2], z = qi[3], w = qi[0], t0 = ti[0], t1 = ti[1], t2 = ti[2];
  for (size_t i = 0; i < n; i++) {
    const double v0 = px[i], v1 = py[i], v2 = pz[i];
    double u0 = y * v2 - z * v1, u1 = z * v0 - x * v2, u2 = x * v1 - y * v0;
    u0 += u0;
    u1 += u1;
    u2 += u2;
    const double c0 = y * u2 - z * u1, c1 = z * u0 - x * u2, c2 = x * u1 - y * u0;
    ox[i] = (float)((v0 + w * u0 + c0) + t0);
    oy[i] = (float)((v1 + w * u1 + c1) + t1);
    oz[i] = (float)((v2 + w * u2 + c2) + t2);
  }
}

}  // namespace

class ReplayEngine {
 public:
  AssocEngine* A = nullptr;
  std::string flag;
  Pose pz;
  CamDev camdev;
  bool biForest = true;  // Object.cc:31 (sticky)
  std::vector<std::unique_ptr<Obj>> objs;
  // map points by id: ids in [0, 2^24) live in an arena of fixed blocks indexed by id
  // (stable addresses, and the points of an object -- ids of one neighbourhood -- sit
  // next to each other, so the host loops over clouds stream instead of chasing
  // pointers); other ids in a map
  static constexpr int kMpBlock = 1024;
  std::vector<std::unique_ptr<MapPt[]>> mp_blocks;
  std::vector<std::unique_ptr<uint8_t[]>> mp_live;
  std::map<int, std::unique_ptr<MapPt>> mps;
  PosSet posset;
  unsigned epoch = 1;  // bumped whenever the pose changes
  void proj_pt(MapPt* p, float& u, float& v) {
    if (p->proj_epoch != epoch) {
      pz.proj(p->pos, p->pu, p->pv);
      p->proj_epoch = epoch;
    }
    u = p->pu;
    v = p->pv;
  }
  MapPt* mp_lookup(int id) {  // existing map point or null
    if (id >= 0 && id < (1 << 24)) {
      const size_t b = (size_t)id / kMpBlock, k = (size_t)id % kMpBlock;
      return b < mp_blocks.size() && mp_live[b] && mp_live[b][k] ? &mp_blocks[b][k] : nullptr;
    }
    auto it = mps.find(id);
    return it == mps.end() ? nullptr : it->second.get();
  }
  MapPt* mappoint(int id) {
    if (id >= 0 && id < (1 << 24)) {
      const size_t b = (size_t)id / kMpBlock, k = (size_t)id % kMpBlock;
      if (b >= mp_blocks.size()) {
        mp_blocks.resize(b + 1);
        mp_live.resize(b + 1);
      }
      if (!mp_blocks[b]) {
        mp_blocks[b].reset(new MapPt[kMpBlock]);
        mp_live[b].reset(new uint8_t[kMpBlock]());
      }
      MapPt* p = &mp_blocks[b][k];
      if (!mp_live[b][k]) {
        mp_live[b][k] = 1;
        p->id = id;
      }
      return p;
    }
    std::unique_ptr<MapPt>& u = mps[id];
    if (!u) {
      u.reset(new MapPt());
      u->id = id;
    }
    return u.get();
  }
  void mp_erase(int id) {  // forget a map point (a discarded look-ahead's own creation)
    if (id >= 0 && id < (1 << 24)) {
      const size_t b = (size_t)id / kMpBlock, k = (size_t)id % kMpBlock;
      if (b < mp_blocks.size() && mp_live[b] && mp_live[b][k]) {
        mp_live[b][k] = 0;
        mp_blocks[b][k] = MapPt();
      }
      return;
    }
    mps.erase(id);
  }
  std::vector<std::unique_ptr<Det>> dets;
  bool ini = false;
  long ini_frame = 0;
  unsigned long cur = 0;
  // GPU staging: pinned host buffers and device mirrors, so every launch is
  // one packed upload + one download on the association stream
  unsigned char *h_in = nullptr, *d_in = nullptr, *h_out = nullptr, *d_out = nullptr;
  size_t cap_in = 0, cap_out = 0;
  // per frame NP results: (det index, object index) -> stats at an object
  // version; an object's version is bumped each time it is modified
  struct NpEntry {
    eao_np_stats st;
    int ver;
  };
  std::map<std::pair<int, int>, NpEntry> np_cache;
  std::vector<int> over;          // object version within this frame
  std::vector<Det*> kept_cur;     // this frame's kept detections, in association order
  int kept_pos = -1;              // the detection being associated
  bool cur_np_done = false;       // ... and whether its NP step has read the cache
  // wall-clock profile (us): frame, local mapping, iForest flushes, NP, rects
  double prof[60] = {0};
  double frame_t0 = 0;  // now_us() at the current frame's begin (prof[58])
  int phase = 0;
  // development trace (EAO_REPLAY_TRACE=<file>): host events on the steady clock (ns, the
  // clock rocprofv3's kernel timestamps use), written at destruction -- tools/replay_timeline.py
  struct TraceEv {
    int64_t t;
    int32_t ev, a, b, c;
  };
  std::vector<TraceEv> trace;
  const char* trace_path = std::getenv("EAO_REPLAY_TRACE");
  void tr(int ev, int a = 0, int b = 0, int c = 0) {
    if (!trace_path) return;
    trace.push_back({std::chrono::duration_cast<std::chrono::nanoseconds>(
                         std::chrono::steady_clock::now().time_since_epoch()).count(), ev, a, b, c});
  }
  static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }
  struct Tick {
    double* acc;
    double t0;
    Tick(double* a) : acc(a), t0(now_us()) {}
    ~Tick() { *acc += now_us() - t0; }
  };

  // isolation forests run asynchronously in batches: every pending object not
  // yet launched is launched together (kick) before the host blocks on any
  // other GPU result and whenever a pending object's points are needed; an
  // object's outliers are erased (complete) the first time its points are read
  static constexpr int kIfBatches = 8, kIfStreams = 4;
  // a device-form record's readiness for the exchange: the Done it was recorded on and, on HSA
  // lanes, the producer lane's ready flag and the value k_publish stores there after it
  struct ExRef {
    int lane = -1;  // ready flag index (forest lanes 0..kIfStreams-1, the frame start's lane kIfStreams)
    uint64_t value = 0;
    int ticket = -1;  // the exchange, once started (Exchanger::start_device)
  };
  struct IfBatch {
    std::vector<Obj*> objs;
    int left = 0;  // objects not yet completed
    // speculative NP pairs evaluated right behind the forest, on the object as
    // it will stand after the erasure: (det index, object index, version)
    std::vector<int> sp_det, sp_obj, sp_ver;  // sp_obj: position in objs
    size_t sp_out = 0;  // byte offset of their stats in h_out
    // launch list (the owned objects), their offsets in the packed clouds
    std::vector<int> lc, loff;
    bool launched = false;
    uint64_t seq = 0;       // launch order (if_seq at the launch)
    unsigned long fid = 0;  // frame of the launch (speculative NP stats belong to it)
    // sharded: the all-gathered outcome, an outlier bit mask per object
    // (mask_off into xres) and the speculative NP stats in sp_* order
    bool xdone = true;
    std::vector<unsigned char> xres;
    std::vector<size_t> mask_off;
    std::vector<eao_np_stats> spst;
    Done done;  // the batch's launches complete (its lane's last packet / event)
    unsigned char *h_in = nullptr, *h_out = nullptr, *d_in = nullptr, *d_out = nullptr;
    size_t cap_in = 0, cap_out = 0;
    // HSA lanes: the packed inputs written by the host straight into device memory through the
    // BAR (bar_alloc), so the batch needs no staging kernel
    unsigned char* bar_in = nullptr;
    size_t cap_bar = 0;
    double* contrib = nullptr;  // [50][max_points]
    // sharded: the per-rank record layout fixed at the launch (mask bytes, speculative
    // pairs, padded record size) and, in the device form, this rank's record in device
    // memory, written by the forest batch's own kernels (k_iforest_sum's masks, np_batch)
    std::vector<size_t> xmb, xnsr;
    size_t xbytes = 0;
    unsigned char* d_x = nullptr;
    size_t cap_x = 0;
    ExRef xr;  // when d_x is complete (HSA lanes: the lane's ready flag value)
  };
  std::vector<IfBatch> ifb;
  // the forest lanes, and the frame start's own lane (HSA form; the HIP form launches the
  // frame start on the engine's stream): HSA queues unless sharded or EAO_HSA_LANES=0
  Lane if_stream[kIfStreams];
  Lane fs_lane;
  // the batch whose launch is the last work queued on each forest stream (-1: other work
  // or none): a launch that waits on that batch alone can queue behind it on its stream
  int if_tail[kIfStreams] = {-1, -1, -1, -1};
  uint64_t if_seq = 0;
  int if_next = 0;
  int pend_err = 0;

  uint64_t xpub[kIfStreams + 1] = {};  // values published so far per lane
  ExRef fs_xr;                          // the frame start's record (d_out)
  // after the launches on HSA lane l (flag index li): zero [zero, zero + bytes) and publish the
  // lane's next flag value; *xr = where the exchange waits for it
  int publish(const Lane& l, int li, void* zero, size_t bytes, ExRef* xr) {
    uint64_t* f = ex ? ex->ready_flag(li) : nullptr;
    if (!f) {
      set_error("replay: no ready flag for the sharded exchange on HSA lanes");
      return EAO_E_STATE;
    }
    xr->lane = li;
    xr->value = ++xpub[li];
    return A->publish(l, zero, bytes, f, xr->value);
  }
  // flag index of a lane of this replay
  int lane_index(const Lane& l) const {
    if (l.q && l.q == fs_lane.q) return kIfStreams;
    for (int k = 0; k < kIfStreams; k++)
      if (l.q && l.q == if_stream[k].q) return k;
    return -1;
  }

  // object sharding (shard.h): the GPU work of object o runs on
  // rank o->id % sworld and its result records are all-gathered
  std::unique_ptr<Exchanger> ex;
  int srank = 0, sworld = 1;
  double xstat[4] = {0};  // exchanges, bytes per rank, us in the exchange
  std::vector<unsigned char> xsend, xrecv;
  int owner(const Obj* o) const { return o->id % sworld; }
  bool mine(const Obj* o) const { return sworld == 1 || owner(o) == srank; }
  // sharded replay: records are exchanged (also at world 1 when an RCCL communicator is
  // set, which runs the exchange path end to end on one device)
  bool sharded() const { return (bool)ex; }
  // device form of the exchange (RCCL): records written and gathered in device memory
  bool xdev() const { return ex && ex->device_form(); }
  // all-gather xsend (padded to `bytes`) into xrecv [sworld][bytes]
  int exchange(size_t bytes) {
    const double t0 = now_us();
    bytes = std::max<size_t>(al16(bytes), 16);
    xsend.resize(bytes, 0);
    xrecv.resize(bytes * sworld);
    int rc = ex->allgather(xsend.data(), xrecv.data(), bytes);
    xstat[0] += 1;
    xstat[1] += (double)bytes;
    xstat[2] += now_us() - t0;
    return rc;
  }
  // device form: this rank's `bytes` at d_send (ready behind `ev`) gathered on the GPU;
  // *recv = the [sworld][bytes] records in pinned host memory
  // Started where the result is read (or, EAO_SHARD_EAGER=1, when the record's launches are
  // enqueued: every rank launches in the same order, so the collectives keep one order); the
  // all-gather waits for the record on the GPU, the host for the gathered copy.
  int exchange_start(const void* d_send, const Done& ev, ExRef& xr, size_t bytes) {
    const double t0 = now_us();
    ExReady rd;
    if (ev.e) {
      rd.ev = ev.e;  // HIP lanes: a GPU-side event wait
    } else if (xr.lane >= 0) {
      rd.flag = ex->ready_flag(xr.lane);  // HSA lanes: a GPU-side wait on the lane's ready flag
      rd.value = xr.value;
    } else if (ev.sig) {
      set_error("replay: an HSA-lane record without its ready flag");
      return EAO_E_STATE;
    }
    int rc = ex->start_device(d_send, rd, bytes, &xr.ticket);
    xstat[0] += 1;
    xstat[1] += (double)bytes;
    xstat[2] += now_us() - t0;
    return rc;
  }
  int exchange_device(const void* d_send, const Done& ev, ExRef& xr, size_t bytes, const unsigned char** recv) {
    if (xr.ticket < 0)
      if (int rc = exchange_start(d_send, ev, xr, bytes)) return rc;
    const double t0 = now_us();
    const int rc = ex->wait_device(xr.ticket, recv);
    xr.ticket = -1;
    xstat[2] += now_us() - t0;
    return rc;
  }

  // forest slots, streams and staging outlive the replay: the next replay on
  // the same engine adopts them (allocation is not per replay)
  Done gpu0;            // frame-start launch completion (spin-waited)
  unsigned char* fs_bar = nullptr;  // the frame start's inputs in device memory (HSA lanes, BAR)
  size_t cap_fs_bar = 0;
  bool rn_dev = false;  // rects_np_launch writes its outputs to d_out (device-form exchange)
  struct Pool {
    std::vector<IfBatch> ifb;
    Lane if_stream[kIfStreams], fs_lane;
    unsigned char* fs_bar = nullptr;
    size_t cap_fs_bar = 0;
    unsigned char *h_in = nullptr, *d_in = nullptr, *h_out = nullptr, *d_out = nullptr;
    size_t cap_in = 0, cap_out = 0;
  };
  static void free_pool(void* v) {
    Pool* p = (Pool*)v;
    ReplayEngine tmp;  // its destructor releases the resources
    tmp.ifb.swap(p->ifb);
    for (int k = 0; k < kIfStreams; k++) tmp.if_stream[k] = p->if_stream[k];
    tmp.fs_lane = p->fs_lane;
    tmp.fs_bar = p->fs_bar;
    tmp.h_in = p->h_in;
    tmp.d_in = p->d_in;
    tmp.h_out = p->h_out;
    tmp.d_out = p->d_out;
    delete p;
  }
  void adopt() {
    if (!A || !A->replay_pool) return;
    Pool* p = (Pool*)A->replay_pool;
    A->replay_pool = nullptr;
    ifb.swap(p->ifb);
    for (IfBatch& b : ifb) {
      b.objs.clear();
      b.left = 0;
      b.xdone = true;
      b.launched = false;
    }
    for (int k = 0; k < kIfStreams; k++) if_stream[k] = p->if_stream[k];
    fs_lane = p->fs_lane;
    fs_bar = p->fs_bar;
    cap_fs_bar = p->cap_fs_bar;
    h_in = p->h_in;
    d_in = p->d_in;
    h_out = p->h_out;
    d_out = p->d_out;
    cap_in = p->cap_in;
    cap_out = p->cap_out;
    delete p;
  }
  ~ReplayEngine() {
    for (const Lane& st : if_stream) (void)lane_sync(st);
    (void)lane_sync(fs_lane);
    if (trace_path && !trace.empty())
      if (FILE* f = std::fopen(trace_path, "ab")) {
        std::fwrite(trace.data(), sizeof(TraceEv), trace.size(), f);
        std::fclose(f);
      }
    done_close(gpu0);
    if (A && !A->replay_pool && !ifb.empty()) {
      Pool* p = new Pool();
      p->ifb.swap(ifb);
      for (int k = 0; k < kIfStreams; k++) {
        p->if_stream[k] = if_stream[k];
        if_stream[k] = Lane();
      }
      p->fs_lane = fs_lane;
      fs_lane = Lane();
      p->fs_bar = fs_bar;
      p->cap_fs_bar = cap_fs_bar;
      fs_bar = nullptr;
      p->h_in = h_in;
      p->d_in = d_in;
      p->h_out = h_out;
      p->d_out = d_out;
      p->cap_in = cap_in;
      p->cap_out = cap_out;
      h_in = d_in = h_out = d_out = nullptr;
      A->replay_pool = p;
      A->replay_pool_free = &ReplayEngine::free_pool;
    }
    for (IfBatch& sl : ifb) {
      done_close(sl.done);
      bar_free(sl.bar_in);
      if (sl.h_in) (void)hipHostFree(sl.h_in);
      if (sl.h_out) (void)hipHostFree(sl.h_out);
      if (sl.d_in) (void)hipFree(sl.d_in);
      if (sl.d_out) (void)hipFree(sl.d_out);
      if (sl.d_x) (void)hipFree(sl.d_x);
      if (sl.contrib) (void)hipFree(sl.contrib);
    }
    for (Lane& st : if_stream) lane_close(st);
    lane_close(fs_lane);
    bar_free(fs_bar);  // (null when handed to the engine's pool above)
    if (h_in) (void)hipHostFree(h_in);
    if (h_out) (void)hipHostFree(h_out);
    if (d_in) (void)hipFree(d_in);
    if (d_out) (void)hipFree(d_out);
  }

  static size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }
  // capacity of the staging buffers (the stream is idle between launches)
  int stage(size_t in_bytes, size_t out_bytes) {
    if (in_bytes > cap_in) {
      const size_t c = std::max(in_bytes, 2 * cap_in);
      if (h_in) (void)hipHostFree(h_in);
      if (d_in) (void)hipFree(d_in);
      h_in = d_in = nullptr;
      cap_in = 0;
      EAO_HIP_CHECK(hipHostMalloc((void**)&h_in, c, 0));
      EAO_HIP_CHECK(hipMalloc((void**)&d_in, c));
      cap_in = c;
    }
    if (out_bytes > cap_out) {
      const size_t c = std::max(out_bytes, 2 * cap_out);
      if (h_out) (void)hipHostFree(h_out);
      if (d_out) (void)hipFree(d_out);
      h_out = d_out = nullptr;
      cap_out = 0;
      EAO_HIP_CHECK(hipHostMalloc((void**)&h_out, c, 0));
      EAO_HIP_CHECK(hipMalloc((void**)&d_out, c));
      cap_out = c;
    }
    return EAO_OK;
  }

  // ---------------------------------------------------------------- object lines + yaw (E14)
  std::vector<std::vector<float>> staged_lines;  // eao_replay_lines, one set per frame
  size_t staged_next = 0;

  static bool yaw_class(int c) { return c == 73 || c == 64 || c == 65 || c == 66 || c == 56; }
  bool yaw_on() const { return flag != "None" && flag != "iForest"; }

  // merge_break_lines (detect_3d_cuboid/object_3d_util.cpp:349-436; fast_RemoveRow
  // matrix_utils.cpp:201-205), thresholds of Tracking.cc:2515-2521
  static void merge_lines(std::vector<double>& L, std::vector<double>& ang) {
    const double dist_th = 20, ath = 5 / 180.0 * M_PI, len_th = 30;
    int total = (int)L.size() / 4, counter = 0;
    bool can = true;
    auto nrm = [](double x, double y) { return std::sqrt(x * x + y * y); };
    while (can && counter < 500) {
      counter++;
      can = false;
      ang.resize(total);
      for (int i = 0; i < total; i++) ang[i] = std::atan2(L[4 * i + 3] - L[4 * i + 1], L[4 * i + 2] - L[4 * i]);
      for (int s1 = 0; s1 < total - 1 && !can; s1++)
        for (int s2 = s1 + 1; s2 < total; s2++) {
          const double diff = std::abs(ang[s1] - ang[s2]);
          if (!(std::min(diff, M_PI - diff) < ath)) continue;
          const double* A = &L[4 * s1];
          const double* B = &L[4 * s2];
          if (!(nrm(A[2] - B[0], A[3] - B[1]) < dist_th || nrm(B[2] - A[0], B[3] - A[1]) < dist_th)) continue;
          const double* st = A[0] < B[0] ? A : B;
          const double* en = A[2] > B[2] ? A : B;
          const double s0 = st[0], s1y = st[1], e0 = en[2], e1 = en[3];
          const double t = std::abs(ang[s1] - std::atan2(e1 - s1y, e0 - s0));
          if (!(std::min(t, M_PI - t) < ath)) continue;
          L[4 * s1] = s0;
          L[4 * s1 + 1] = s1y;
          L[4 * s1 + 2] = e0;
          L[4 * s1 + 3] = e1;
          for (int c = 0; c < 4; c++) L[4 * s2 + c] = L[4 * (total - 1) + c];
          total--;
          can = true;
          break;
        }
    }
    int w = 0;
    for (int i = 0; i < total; i++) {
      if (!(nrm(L[4 * i + 2] - L[4 * i], L[4 * i + 3] - L[4 * i + 1]) > len_th)) continue;
      for (int c = 0; c < 4; c++) L[4 * w + c] = L[4 * i + c];
      w++;
    }
    L.resize(4 * w);
  }

  // Tracking::AssociateObjAndLines (Tracking.cc:2472-2527) for the detections whose
  // lines SampleObjYaw can read (yaw-sampled classes); the frame's staged line set.
  // `took` (the look-ahead): set when a staged set was consumed -- a discarded look-ahead steps
  // staged_next back over it, so the staged sets are not cleared while the look-ahead holds one
  void associate_lines(const std::vector<Det*>& o2, bool* took = nullptr) {
    const std::vector<float>* fl = staged_next < staged_lines.size() ? &staged_lines[staged_next] : nullptr;
    if (fl) staged_next++;
    if (fl && took) *took = true;
    std::vector<double> all, in, ang;
    if (fl && yaw_on()) {
      all.assign(fl->begin(), fl->end());
      for (size_t i = 0; i + 3 < all.size(); i += 4)  // align_left_right_edges
        if (all[i + 2] < all[i]) {
          std::swap(all[i], all[i + 2]);
          std::swap(all[i + 1], all[i + 3]);
        }
      for (Det* f : o2) {
        if (!yaw_class(f->cls)) continue;
        const double l = std::max(0.0, f->bx - 15.0), r = (double)std::min(pz.cols, f->bx + f->bw + 15);
        const double t = std::max(0.0, f->by - 15.0), b = (double)std::min(pz.rows, f->by + f->bh + 15);
        in.clear();
        for (size_t i = 0; i + 3 < all.size(); i += 4) {
          const double* e = &all[i];
          if (l <= e[0] && e[0] <= r && t <= e[1] && e[1] <= b && l <= e[2] && e[2] <= r && t <= e[3] && e[3] <= b)
            in.insert(in.end(), e, e + 4);
        }
        merge_lines(in, ang);
        const int n = (int)in.size() / 4;
        f->line_deg.resize(n);
        for (int i = 0; i < n; i++) {
          const float a = (float)std::atan2(in[4 * i + 3] - in[4 * i + 1], in[4 * i + 2] - in[4 * i]);
          f->line_deg[i] = (double)(a * 180) / M_PI;
        }
      }
    }
    if (!took) release_staged_lines();
  }
  // all staged sets consumed (and none held by a look-ahead): drop them
  void release_staged_lines() {
    if (staged_next == staged_lines.size() && !staged_lines.empty()) {
      staged_lines.clear();
      staged_next = 0;
    }
  }

  // Tracking::SampleObjYaw (Tracking.cc:2624-2871) with WorldToImg (:2602-2620)
  void sample_yaw(Obj* o, const float* Tcw) {
    Pose pv = pz;  // WorldToImg under the pose of the sampled frame
    std::memcpy(pv.T, Tcw, sizeof(pv.T));
    const std::vector<double>& L = o->frames.back()->line_deg;
    const int nAll = (int)L.size();
    int numMax = 0;
    float fError = 0.0f, fErrorYaw = 0.0f, sampleYaw = 0.0f;
    float ctr[3], rel[8][3];
    for (int a = 0; a < 3; a++) ctr[a] = (float)o->center_c[a];
    for (int k = 0; k < 8; k++)
      for (int a = 0; a < 3; a++) rel[k][a] = (float)o->corner_w[k][a] - ctr[a];
    static const int ea[3] = {4, 5, 1}, eb[3] = {5, 6, 5};  // 5->6, 6->7, 2->6 (1-based corners)
    for (int i = 0; i < 30; i++) {
      const float yaw = i < 15 ? (float)((0.0 - i * 3.0) / 180.0 * M_PI) : (float)((0.0 + (i - 15) * 3.0) / 180.0 * M_PI);
      const float pitch = 0.0f, roll = 0.0f;
      const float cp = std::cos(pitch), sp = std::sin(pitch), sr = std::sin(roll), cr = std::cos(roll);
      // sin/cos of the sampled yaw correctly rounded via double (Q26): a constant-folded
      // sinf and a libm sinf may differ by an ulp
      const float sy = (float)std::sin((double)yaw), cy = (float)std::cos((double)yaw);
      const float R[3][3] = {{cp * cy, (sr * sp * cy) - (cr * sy), (cr * sp * cy) + (sr * sy)},
                             {cp * sy, (sr * sp * sy) + (cr * cy), (cr * sp * sy) - (sr * cy)},
                             {-sp, sr * cp, cr * cp}};
      float px[8], py[8];
      for (int k = 0; k < 8; k++) {
        if (k == 0 || k == 2 || k == 3 || k == 7) continue;  // only corners 2, 5, 6, 7 are read
        float w[3];
        for (int r = 0; r < 3; r++) {
          const float d = R[r][0] * rel[k][0] + R[r][1] * rel[k][1] + R[r][2] * rel[k][2];
          w[r] = (float)((double)d + (double)ctr[r]);
        }
        pv.proj(w, px[k], py[k]);
      }
      double adeg[3];
      float len[3];
      for (int e = 0; e < 3; e++) {
        const int a = ea[e], b = eb[e];
        const float ang = px[b] > px[a] ? std::atan2(py[b] - py[a], px[b] - px[a]) : std::atan2(py[a] - py[b], px[a] - px[b]);
        adeg[e] = (double)(ang * 180) / M_PI;
        len[e] = std::sqrt((py[b] - py[a]) * (py[b] - py[a]) + (px[b] - px[a]) * (px[b] - px[a]));
      }
      const float mn = std::min(std::min(len[0], len[1]), len[2]);
      float error = 0.0f, errorYaw = 0.0f;
      int num = 0;
      const float th = 5.0f;
      for (int li = 0; li < nAll; li++) {
        const float d1 = (float)std::abs(L[li] - adeg[0]);
        const float d2 = (float)std::abs(L[li] - adeg[1]);
        const float d3 = (float)std::abs(L[li] - adeg[2]);
        if (o->cls == 56) {
          if ((d2 < th) || (d3 < th)) num++;
          if (d1 < th) num += 3;
          continue;
        }
        if (mn == len[0]) {
          if ((d2 < th) || (d3 < th)) {
            num++;
            if (d2 < th) error += d2;
            if (d3 < th) error += d3;
          }
          errorYaw += std::min(d2, d3);
        }
        if (mn == len[1]) {
          if ((d1 < th) || (d3 < th)) {
            num++;
            if (d1 < th) error += d1;
            if (d3 < th) error += d3;
          }
          errorYaw += std::min(d3, d1);
        }
        if (mn == len[2]) {
          if ((d1 < th) || (d2 < th)) {
            num++;
            if (d1 < th) error += d1;
            if (d2 < th) error += d2;
          }
          errorYaw += std::min(d2, d1);
        }
      }
      if (num == 0) {
        num = 1;
        errorYaw = 10.0f;
      }
      if (num > numMax) {
        numMax = num;
        sampleYaw = yaw;
        fError = error;
        fErrorYaw = (float)((double)(errorYaw / (float)num) / 10.0);
      }
    }
    float fScore = (float)((double)((float)numMax / (float)nAll) * (1.0 - 0.1 * (double)fErrorYaw));
    if (std::isinf(fScore)) fScore = 0.0f;
    const std::array<float, 5> v = {sampleYaw, 1.0f, fScore, fError, fErrorYaw};
    bool fresh = true;
    for (auto& row : o->angles)
      if (row[0] == v[0]) {
        row[1] += 1.0f;
        for (int q = 2; q < 5; q++) row[q] = v[q] * (1 / row[1]) + row[q] * (1 - 1 / row[1]);
        fresh = false;
      }
    if (fresh) o->angles.push_back(v);
    std::sort(o->angles.begin(), o->angles.end(),  // VIC, index = 1 (Tracking.cc:63-68)
              [](const std::array<float, 5>& l, const std::array<float, 5>& r) { return l[1] > r[1]; });
    int best = 0;
    float best_score = 0;
    for (int i = 0; i < std::min(3, (int)o->angles.size()); i++)
      if (o->angles[i][2] >= best_score) {
        best_score = o->angles[i][2];
        best = i;
      }
    o->rotY = o->angles[best][0];
    o->err_par = o->angles[best][3];
    o->err_yaw = o->angles[best][4];
  }

  // ---------------------------------------------------------------- cuboid / stats
  void update_pose(Obj* o) {  // Object_Map::UpdateObjPose, Object.cc:2193-2248
    const float cp = std::cos(o->rotP), sp = std::sin(o->rotP), sr = std::sin(o->rotR),
                cr = std::cos(o->rotR), sy = std::sin(o->rotY), cy = std::cos(o->rotY);
    const float Rf[3][3] = {{cp * cy, (sr * sp * cy) - (cr * sy), (cr * sp * cy) + (sr * sy)},
                            {cp * sy, (sr * sp * sy) + (cr * cy), (cr * sp * sy) - (sr * cy)},
                            {-sp, sr * cp, cr * cp}};
    double R[3][3];
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) R[a][b] = (double)Rf[a][b];
    quat_from_R(R, o->q);
    for (int a = 0; a < 3; a++) o->t[a] = (double)(float)o->center_c[a];
    const double I[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    quat_from_R(I, o->qn);
    o->tn[0] = (double)o->center[0];
    o->tn[1] = (double)(float)o->center_c[1];
    o->tn[2] = (double)o->center[2];
  }

  // Object_Map::ComputeMeanAndStandard, Object.cc:967-1198 (min/max replace the sorts)
  // ComputeMeanAndStandard scratch: the object's positions gathered once per call (SoA), and
  // their images under the inverse cuboid pose
  std::vector<float> ms_p[3], ms_t[3];
  // mean_std's input positions when the caller has them in order already (big_to_small over an
  // object's cached ones): x, y, z blocks of the list's length, no point bad
  const float* ms_in = nullptr;
  std::vector<float> bts_p;
  uint64_t pt_epoch = 1;  // bumped whenever a map point's position or bad flag changes
  // a point that changes marks the objects it voted for: every object that holds a point got its
  // vote first (vote / vote_insert before each pts.push_back) and votes are never withdrawn
  void point_changed(MapPt* p) {
    p->ver = ++pt_epoch;
    for (auto& v : p->votes)
      if ((size_t)v.first < objs.size()) objs[v.first]->pt_chg = pt_epoch;
  }
  bool points_unchanged(const Obj* o, uint64_t since) const {
    if (o->pt_chg > since) return false;
    if (g_ms_verify)
      for (const MapPt* p : o->pts)
        if (p->ver > since) {
          fprintf(stderr, "eao: point %d of object %d changed unmarked\n", p->id, o->id);
          abort();
        }
    return true;
  }
  // mean_std(o) with exactly the inputs of its last call: it would write the values o holds now
  bool mean_std_same(const Obj* o) const {
    if (!g_ms_memo || o->ms_epoch == ~0ull || o->pts.size() != o->ms_pts.size() ||
        o->frames.size() * 3 != o->ms_fp.size() || o->rotY != o->ms_rot[0] || o->rotP != o->ms_rot[1] ||
        o->rotR != o->ms_rot[2])
      return false;
    for (int a = 0; a < 3; a++)  // the centre update_pose starts from (frames >= 5): a fixed point
      if (o->frames.size() >= 5 && !(o->center_c[a] == o->ms_cc_out[a] && o->ms_cc_in[a] == o->ms_cc_out[a]))
        return false;
    if (!o->pts.empty() && std::memcmp(o->pts.data(), o->ms_pts.data(), sizeof(MapPt*) * o->pts.size()) != 0)
      return false;
    if (!points_unchanged(o, o->ms_epoch)) return false;
    for (size_t k = 0; k < o->frames.size(); k++) {
      const float* fp = o->frames[k]->P();
      if (std::memcmp(fp, &o->ms_fp[3 * k], sizeof(float) * 3) != 0) return false;
    }
    return true;
  }
  void mean_std(Obj* o) {
    if (mean_std_same(o)) {
      prof[27] += 1;
      return;
    }
    double cc_in[3];
    for (int a = 0; a < 3; a++) cc_in[a] = o->center_c[a];
    o->ms_epoch = ~0ull;
    struct Memo {  // the inputs of this call, recorded on every return
      Obj* o;
      const double* cc;
      const uint64_t ep;
      ~Memo() {
        o->ms_epoch = ep;
        o->ms_pts = o->pts;
        o->ms_fp.resize(3 * o->frames.size());
        for (size_t k = 0; k < o->frames.size(); k++) std::memcpy(&o->ms_fp[3 * k], o->frames[k]->P(), sizeof(float) * 3);
        o->ms_rot[0] = o->rotY;
        o->ms_rot[1] = o->rotP;
        o->ms_rot[2] = o->rotR;
        for (int a = 0; a < 3; a++) {
          o->ms_cc_in[a] = cc[a];
          o->ms_cc_out[a] = o->center_c[a];
        }
      }
    } memo{o, cc_in, pt_epoch};
    double T0 = now_us();
    for (int a = 0; a < 3; a++) o->sum[a] = 0;
    const size_t n0 = o->pts.size();
    for (int a = 0; a < 3; a++)
      if (ms_p[a].size() < n0) {
        ms_p[a].resize(n0 + n0 / 2 + 64);
        ms_t[a].resize(n0 + n0 / 2 + 64);
      }
    float* px = ms_p[0].data();
    float* py = ms_p[1].data();
    float* pz = ms_p[2].data();
    size_t w = 0;
    if (ms_in) {  // the same sums in the same order (float, per axis), from contiguous positions
      for (int a = 0; a < 3; a++) {
        const float* in = ms_in + a * n0;
        float* out = ms_p[a].data();
        float sa = 0;
        for (size_t i = 0; i < n0; i++) {
          sa += in[i];
          out[i] = in[i];
        }
        o->sum[a] = sa;
      }
      w = n0;
    } else {
      for (size_t i = 0; i < n0; i++) {
        MapPt* p = o->pts[i];
        if (p->bad) continue;
        for (int a = 0; a < 3; a++) o->sum[a] += p->pos[a];
        px[w] = p->pos[0];
        py[w] = p->pos[1];
        pz[w] = p->pos[2];
        o->pts[w++] = p;
      }
      o->pts.resize(w);
    }
    const size_t n = o->pts.size();
    o->ms_pos.resize(3 * n);  // cached for the next call over this list (big_to_small)
    std::memcpy(o->ms_pos.data(), px, sizeof(float) * n);
    std::memcpy(o->ms_pos.data() + n, py, sizeof(float) * n);
    std::memcpy(o->ms_pos.data() + 2 * n, pz, sizeof(float) * n);
    const float sc = (float)(1. / (double)n);
    for (int a = 0; a < 3; a++) o->center[a] = o->sum[a] * sc + 0.0f;
    float s2[3] = {0, 0, 0};
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    {
      const float c0 = o->center[0], c1 = o->center[1], c2 = o->center[2];
      for (size_t i = 0; i < n; i++) {  // the three sums in point order (float, as the reference)
        s2[0] += (px[i] - c0) * (px[i] - c0);
        s2[1] += (py[i] - c1) * (py[i] - c1);
        s2[2] += (pz[i] - c2) * (pz[i] - c2);
      }
      for (int a = 0; a < 3; a++) minmax_scan(ms_p[a].data(), n, mn[a], mx[a]);
    }
    for (int a = 0; a < 3; a++) o->sd[a] = std::sqrt(s2[a] / (float)n);
    double T1 = now_us(); prof[32] += T1 - T0;
    if (n == 0) return;
    float c2[3] = {0, 0, 0};
    for (Det* f : o->frames) {
      const float* fp = f->P();
      for (int a = 0; a < 3; a++) c2[a] += (fp[a] - o->center[a]) * (fp[a] - o->center[a]);
    }
    for (int a = 0; a < 3; a++) o->csd[a] = std::sqrt(c2[a] / (float)o->frames.size());
    static const int cx[8] = {0, 1, 1, 0, 0, 1, 1, 0}, cy[8] = {0, 0, 1, 1, 0, 0, 1, 1},
                     cz[8] = {0, 0, 0, 0, 1, 1, 1, 1};
    if (o->frames.size() < 5) {
      o->center_c[0] = (mx[0] + mn[0]) / 2;
      o->center_c[1] = (mx[1] + mn[1]) / 2;
      o->center_c[2] = (mx[2] + mn[2]) / 2;
      o->xmn = mn[0]; o->xmx = mx[0];
      o->ymn = mn[1]; o->ymx = mx[1];
      o->zmn = mn[2]; o->zmx = mx[2];
      o->lenth = mx[0] - mn[0];
      o->width = mx[1] - mn[1];
      o->height = mx[2] - mn[2];
    }
    update_pose(o);
    float omn[3] = {INFINITY, INFINITY, INFINITY}, omx[3] = {-INFINITY, -INFINITY, -INFINITY};
    double qi[4], ti[3];  // pose inverse, identical for every point
    double T2 = now_us(); prof[33] += T2 - T1; prof[36] += n;
    se3_inverse(o->q, o->t, qi, ti);
    se3_batch(qi, ti, n, px, py, pz, ms_t[0].data(), ms_t[1].data(), ms_t[2].data());
    for (int a = 0; a < 3; a++) minmax_scan(ms_t[a].data(), n, omn[a], omx[a]);
    double T3 = now_us(); prof[34] += T3 - T2;
    for (int k = 0; k < 8; k++) {
      const double v[3] = {cx[k] ? omx[0] : omn[0], cy[k] ? omx[1] : omn[1], cz[k] ? omx[2] : omn[2]};
      se3_apply(o->q, o->t, v, o->corner[k]);
      se3_apply(o->qn, o->tn, v, o->corner_w[k]);
    }
    o->lenth = omx[0] - omn[0];
    o->width = omx[1] - omn[1];
    o->height = omx[2] - omn[2];
    for (int a = 0; a < 3; a++) o->center_c[a] = (o->corner[1][a] + o->corner[7][a]) / 2;
    update_pose(o);
    float rm = 0.0f;
    for (int k = 0; k < 8; k++) {
      float d[3];
      for (int a = 0; a < 3; a++) d[a] = o->center[a] - (float)o->corner[k][a];
      rm = std::max(rm, std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]));
    }
    o->rmax = rm;
    float dis = 0;
    for (Det* f : o->frames) {
      const float* fp = f->P();
      float e[3];
      for (int a = 0; a < 3; a++) e[a] = (fp[a] - o->center[a]) * (fp[a] - o->center[a]);
      dis += std::sqrt(e[0] + e[1] + e[2]);
    }
    o->csd_all = std::sqrt(dis / (float)o->frames.size());
    prof[35] += now_us() - T3;
  }

  bool iforest_applies(const Obj* o) const {
    return biForest && !(o->cls == 75 || o->cls == 64 || o->cls == 65) && o->pts.size() >= 30;
  }

  // Object_Map::IsolationForestDeleteOutliers (Object.cc:1202-1309), split in
  // a batched launch and a per-object completion (erase the outliers in list
  // order, Q8, then ComputeMeanAndStandard for pending 2)
  int if_init() {
    ifb.resize(kIfBatches);
    for (IfBatch& b : ifb)
      if (!b.contrib) EAO_HIP_CHECK(hipMalloc((void**)&b.contrib, sizeof(double) * 50 * (size_t)A->max_points));
    return lanes_init();
  }
  // the association is the latency-bound chain of the step: its launches go to lanes of the
  // highest priority (extraction work queued elsewhere cannot delay them), HSA queues fed with
  // AQL packets directly (hsa_lane.h) unless the replay is sharded (RCCL waits on HIP events)
  // or EAO_HSA_LANES=0. Lanes adopted from a previous replay of the other kind are replaced.
  bool lanes_hsa = false;
  int lanes_init() {
    // sharded replays too: the host form waits on the lanes' markers, the device form's RCCL
    // stream on the lanes' ready flags (EAO_SHARD_HSA=0: HIP streams, A/B)
    const bool want = (!sharded() || (g_shard_hsa && (!xdev() || ex->ready_flag(0)))) && hsa_lanes_available(A->dev);
    if (if_stream[0].s || if_stream[0].q) {
      lanes_hsa = if_stream[0].hsa();  // adopted from the previous replay on this engine
      if (lanes_hsa == want) return EAO_OK;
      for (Lane& l : if_stream) lane_close(l);
      lane_close(fs_lane);
      for (IfBatch& b : ifb) done_close(b.done);
      done_close(gpu0);
    }
    lanes_hsa = false;
    if (want) {  // HSA queues are a per-process hardware resource: without them, HIP streams
      if (lanes_open(if_stream, kIfStreams, true, A->dev) == EAO_OK && lanes_open(&fs_lane, 1, true, A->dev) == EAO_OK) {
        lanes_hsa = true;
        return EAO_OK;
      }
      for (Lane& l : if_stream) lane_close(l);
      lane_close(fs_lane);
    }
    return lanes_open(if_stream, kIfStreams, false, A->dev);
  }
  int resolve_trivial(Obj* o) {  // pending objects the forest does not apply to
    if (o->pending == 2) mean_std(o);
    o->pending = 0;
    return EAO_OK;
  }
  // launch every pending, not yet launched object (one or more batches)
  int kick() {
    Tick tk(&prof[18]);
    std::vector<Obj*> todo;
    double tscan = now_us();
    for (auto& up : objs) {
      Obj* o = up.get();
      if (!o->pending || o->slot >= 0) continue;
      if (!iforest_applies(o)) {
        resolve_trivial(o);
        continue;
      }
      if ((int)o->pts.size() > IF_MAXN) {
        set_error("replay: object exceeds the isolation-forest capacity");
        return EAO_E_CAPACITY;
      }
      todo.push_back(o);
    }
    prof[22] += now_us() - tscan;
    if (todo.empty()) return EAO_OK;
    if (ifb.empty()) {
      int rc = if_init();
      if (rc) return rc;
    }
    size_t i = 0;
    while (i < todo.size()) {
      int k = -1;
      for (int t = 0; t < kIfBatches; t++) {
        const int c = (if_next + t) % kIfBatches;
        if (ifb[c].left == 0) {
          k = c;
          break;
        }
      }
      if (k < 0) {  // every batch in flight: retire the oldest
        Tick tr(&prof[21]);
        prof[20] += 1;
        k = if_next;
        std::vector<Obj*> os = ifb[k].objs;
        for (Obj* o : os)
          if (o->slot == k) {
            int rc = complete_forest(o);
            if (rc) return rc;
          }
      }
      if_next = (k + 1) % kIfBatches;
      IfBatch& b = ifb[k];
      b.fid = cur;
      b.objs.clear();
      b.sp_det.clear();
      b.sp_obj.clear();
      b.sp_ver.clear();
      int tot = 0;
      for (; i < todo.size() && (int)b.objs.size() < A->max_clouds; i++) {
        const int n = (int)todo[i]->pts.size();
        if (!b.objs.empty() && tot + n > A->max_points) break;
        b.objs.push_back(todo[i]);
        tot += n;
      }
      const int nb = (int)b.objs.size();
      {  // capacity over the whole batch, not only the owned objects: every rank of a
         // sharded replay must reach the same verdict (no rank left waiting in an exchange)
        int maxN_all = 0;
        for (Obj* o : b.objs) maxN_all = std::max(maxN_all, (int)o->pts.size());
        if (!A->iforest_fits(maxN_all, maxN_all / 2)) {
          set_error("replay: object exceeds the isolation-forest capacity");
          return EAO_E_CAPACITY;
        }
      }
      Tick tpk(&prof[23]);
      // speculative NP: every later detection of this frame that will run the
      // NP test against these objects (same class, >= 20 points, Object.cc:255-339)
      std::vector<Det*> sdets;
      std::vector<int> sdoff, sdz;
      for (int c = 0; c < nb; c++) {
        Obj* o = b.objs[c];
        if (flag == "NA" || flag == "IoU" || o->bad) continue;
        const int q0 = std::max(kept_pos + (cur_np_done ? 1 : 0), 0);
        for (size_t q = (size_t)q0; q < kept_cur.size(); q++) {
          Det* f = kept_cur[q];
          if (f->cls != o->cls || f->pts.size() < 20) continue;
          b.sp_det.push_back(f->index);
          b.sp_obj.push_back(c);  // batch position until the launch list is known
          b.sp_ver.push_back(over[o->id]);
          sdz.push_back((int)q);
        }
      }
      // launch list: the batch's objects this rank owns (all of them unsharded),
      // packed at their own offsets; the speculative pairs of those objects
      b.lc.clear();
      b.loff.assign(nb, -1);
      int np = 0, maxN = 0;
      for (int c = 0; c < nb; c++) {
        if (!mine(b.objs[c])) continue;
        b.lc.push_back(c);
        b.loff[c] = np;
        np += (int)b.objs[c]->pts.size();
        maxN = std::max(maxN, (int)b.objs[c]->pts.size());
      }
      std::vector<int> lsp;
      int nfp = 0, max_olen = 0;
      for (size_t q = 0; q < b.sp_obj.size(); q++) {
        if (!mine(b.objs[b.sp_obj[q]])) continue;
        lsp.push_back((int)q);
        Det* f = kept_cur[sdz[q]];
        int di = -1;
        for (size_t z = 0; z < sdets.size(); z++)
          if (sdets[z] == f) di = (int)z;
        if (di < 0) {
          di = (int)sdets.size();
          sdets.push_back(f);
          sdoff.push_back(nfp);
          nfp += (int)f->pts.size();
        }
        sdz[q] = di;
        max_olen = std::max(max_olen, (int)b.objs[b.sp_obj[q]]->pts.size());
      }
      const int nl = (int)b.lc.size(), ns = (int)lsp.size();
      for (int c = 0; c < nb; c++) b.objs[c]->slot = k;
      b.left = nb;
      if (b.xr.ticket >= 0) {  // the slot's previous exchange, started but never read: drained
        const unsigned char* r = nullptr;
        if (int rc = ex->wait_device(b.xr.ticket, &r)) return rc;
        b.xr = ExRef();
      }
      b.xdone = !sharded();
      b.launched = nl > 0;
      if (sharded()) {
        // the record every rank all-gathers for this batch: per owned object an outlier
        // bit mask, then (from the next 16-byte boundary) the owned speculative NP stats;
        // one padded size for all ranks
        b.xmb.assign(sworld, 0);
        b.xnsr.assign(sworld, 0);
        for (int c = 0; c < nb; c++) b.xmb[owner(b.objs[c])] += (b.objs[c]->pts.size() + 7) / 8;
        for (size_t q = 0; q < b.sp_obj.size(); q++) b.xnsr[owner(b.objs[b.sp_obj[q]])]++;
        b.xbytes = 0;
        for (int r = 0; r < sworld; r++) b.xbytes = std::max(b.xbytes, al16(b.xmb[r]) + sizeof(eao_np_stats) * b.xnsr[r]);
        b.xbytes = std::max<size_t>(al16(b.xbytes), 16);
        if (xdev() && b.xbytes > b.cap_x) {
          if (b.d_x) (void)hipFree(b.d_x);
          b.d_x = nullptr;
          const size_t c = std::max(b.xbytes, 2 * b.cap_x);
          b.cap_x = 0;  // raised only once the allocation exists
          EAO_HIP_CHECK(hipMalloc((void**)&b.d_x, c));
          b.cap_x = c;
        }
        if (xdev() && !b.launched) {  // nothing owned: an empty record, ready behind b.ev
          const Lane& st = if_stream[k % kIfStreams];
          if_tail[k % kIfStreams] = -1;
          b.xr = ExRef();
          if (st.hsa()) {
            if (int rc = publish(st, k % kIfStreams, b.d_x, b.xbytes, &b.xr)) return rc;
          } else {
            EAO_HIP_CHECK(hipMemsetAsync(b.d_x, 0, b.xbytes, st.s));
          }
          if (int rc = lane_record(st, b.done)) return rc;
          if (g_shard_eager)
            if (int rc = exchange_start(b.d_x, b.done, b.xr, b.xbytes)) return rc;
        }
      }
      if (!b.launched) continue;
      // in: forest meta [3 nl] | object points [3 np] | object valid [np] | NP meta [4 ns] | th [ns] |
      //     score pointers [ns] | frame points [3 nfp] | frame valid [nfp]
      // out (host): scores [np] doubles | NP stats [ns]; device: scores [np] for the NP kernels
      // (the speculative pairs here, the next frame start's rects / pairs, frame_start_gpu)
      const size_t o_pts = al16(sizeof(int) * 3 * nl);
      const size_t o_oval = o_pts + sizeof(float) * 3 * (size_t)np;
      const size_t o_spm = al16(o_oval + np);
      const size_t o_th = o_spm + sizeof(int) * 4 * ns;
      const size_t o_osp = al16(o_th + sizeof(float) * ns);
      const size_t o_fp = al16(o_osp + sizeof(double*) * ns);
      const size_t o_fval = o_fp + sizeof(float) * 3 * (size_t)nfp;
      // device-form exchange: the mask packing's meta [3 nl] | thresholds [nl] after the rest
      const size_t o_pk = al16(ns ? o_fval + nfp : o_pts + sizeof(float) * 3 * (size_t)np);
      const size_t o_pkth = o_pk + sizeof(int) * 3 * nl;
      const size_t in_bytes = xdev() ? o_pkth + sizeof(float) * nl
                                     : ns ? o_fval + nfp : o_pts + sizeof(float) * 3 * (size_t)np;
      b.sp_out = al16(sizeof(double) * np);
      const size_t out_bytes = b.sp_out + sizeof(eao_np_stats) * ns;
      if (in_bytes > b.cap_in) {
        if (b.h_in) (void)hipHostFree(b.h_in);
        if (b.d_in) (void)hipFree(b.d_in);
        b.h_in = b.d_in = nullptr;
        const size_t c = std::max(in_bytes, 2 * b.cap_in);
        b.cap_in = 0;  // raised only once both allocations exist
        EAO_HIP_CHECK(hipHostMalloc((void**)&b.h_in, c, 0));
        EAO_HIP_CHECK(hipMalloc((void**)&b.d_in, c));
        b.cap_in = c;
      }
      if (out_bytes > b.cap_out) {
        if (b.h_out) (void)hipHostFree(b.h_out);
        if (b.d_out) (void)hipFree(b.d_out);
        b.h_out = b.d_out = nullptr;
        const size_t c = std::max(out_bytes, 2 * b.cap_out);
        b.cap_out = 0;
        EAO_HIP_CHECK(hipHostMalloc((void**)&b.h_out, c, 0));
        EAO_HIP_CHECK(hipMalloc((void**)&b.d_out, c));
        b.cap_out = c;
      }
      if (b.done.e || b.done.sig) {  // the slot's previous launch (completed on its outputs): a late fault surfaces here
        const hipError_t e = done_query(b.done);
        if (e != hipSuccess && e != hipErrorNotReady) EAO_HIP_CHECK(e);
      }
      if (g_sentinel && !sharded()) {  // scores and speculative stats pre-filled (spin_ready)
        fill64(b.h_out, (size_t)np);
        fill32(b.h_out + b.sp_out, (size_t)ns * (sizeof(eao_np_stats) / 4));
      }
      // the packed inputs: pinned host memory staged by k_stage, or (HSA lanes) device memory
      // written here through the BAR -- write-only (a host read of it is an uncached PCIe round trip)
      unsigned char* hin = b.h_in;
      unsigned char* din = b.d_in;
      if (if_stream[k % kIfStreams].hsa() && g_bar_inputs) {
        if (in_bytes > b.cap_bar) {
          // the slot's previous launch may still read the old buffer (its wait can end on the
          // outputs before the kernels retire): it completes before the buffer goes
          if (b.bar_in && (b.done.e || b.done.sig)) EAO_HIP_CHECK(spin_event_plain(b.done));
          const size_t c = std::max(in_bytes, 2 * b.cap_bar);
          bar_free(b.bar_in);
          b.cap_bar = 0;
          b.bar_in = (unsigned char*)bar_alloc(A->dev, c);
          if (b.bar_in) b.cap_bar = c;
        }
        if (b.bar_in) hin = din = b.bar_in;
      }
      int* meta = (int*)hin;
      float* pts = (float*)(hin + o_pts);
      for (int j = 0; j < nl; j++) {
        Obj* o = b.objs[b.lc[j]];
        int w = b.loff[b.lc[j]];
        meta[j] = w;
        meta[nl + j] = (int)o->pts.size();
        meta[2 * nl + j] = (int)o->pts.size() / 2;
        for (MapPt* p : o->pts) {
          std::memcpy(&pts[3 * (size_t)w], p->pos, sizeof(float) * 3);
          if (ns) hin[o_oval + w] = p->bad ? 0 : 1;  // out_point is never set (Q7)
          w++;
        }
      }
      if (ns) {
        int* spm = (int*)(hin + o_spm);
        float* th = (float*)(hin + o_th);
        const double** osp = (const double**)(hin + o_osp);
        float* fpt = (float*)(hin + o_fp);
        uint8_t* fval = hin + o_fval;
        for (size_t z = 0; z < sdets.size(); z++) {
          int w = sdoff[z];
          for (MapPt* p : sdets[z]->pts) {
            std::memcpy(&fpt[3 * (size_t)w], p->pos, sizeof(float) * 3);
            fval[w++] = p->bad ? 0 : 1;
          }
        }
        for (int j = 0; j < ns; j++) {
          const int q = lsp[j], z = sdz[q], c = b.sp_obj[q];
          Obj* o = b.objs[c];
          spm[j] = sdoff[z];
          spm[ns + j] = (int)sdets[z]->pts.size();
          spm[2 * ns + j] = b.loff[c];
          spm[3 * ns + j] = (int)o->pts.size();
          th[j] = o->cls == 62 ? 0.65f : 0.6f;
          osp[j] = (const double*)b.d_out + b.loff[c];  // device scores of this forest
        }
      }
      if (xdev()) {
        int* pk = (int*)(hin + o_pk);
        float* pth = (float*)(hin + o_pkth);
        size_t w = 0;
        for (int j = 0; j < nl; j++) {
          Obj* o = b.objs[b.lc[j]];
          pk[3 * j] = b.loff[b.lc[j]];
          pk[3 * j + 1] = (int)o->pts.size();
          pk[3 * j + 2] = (int)w;
          pth[j] = o->cls == 62 ? 0.65f : 0.6f;
          w += (o->pts.size() + 7) / 8;
        }
      }
      const Lane& st = if_stream[k % kIfStreams];
      b.seq = ++if_seq;
      if_tail[k % kIfStreams] = k;
      prof[2] += 1;
      Tick tl(&prof[19]);
      // compute-queue staging (k_stage), as at the frame start: no DMA-engine hand-off
      if (din == hin)
        lane_bar_written(st, hin + in_bytes - 1);  // flushed before the batch's doorbell
      else if (int rc0 = A->stage_in(din, hin, in_bytes, st))
        return rc0;
      const int* dm = (const int*)din;
      // scores go straight to pinned host memory (a device-to-host copy costs
      // ~35 us of round trip per launch on this box) and, for the speculative
      // NP pairs, to device memory too
      // device-form exchange: the outlier bit masks go into this rank's record from the score kernel
      int rc = A->iforest_batch(nl, (const float*)(din + o_pts), dm, dm + nl, 50, 12345,
                                (const uint32_t*)(dm + 2 * nl), (double*)b.h_out, st, maxN, maxN / 2, np, b.contrib,
                                (double*)b.d_out, xdev() ? (const int*)(din + o_pk) : nullptr,
                                xdev() ? (const float*)(din + o_pkth) : nullptr, xdev() ? b.d_x : nullptr);
      if (rc) return rc;
      if (ns) {
        const int* spm = (const int*)(din + o_spm);
        const float* dfp = (const float*)(din + o_fp);
        // device-form exchange: the stats go straight into this rank's record
        eao_np_stats* sp_dst = xdev() ? (eao_np_stats*)(b.d_x + al16(b.xmb[srank])) : (eao_np_stats*)(b.h_out + b.sp_out);
        rc = A->np_batch(ns, dfp, din + o_fval, spm, spm + ns, (const float*)(din + o_pts), din + o_oval,
                         spm + 2 * ns, spm + 3 * ns, sp_dst, st, max_olen, (const double* const*)(din + o_osp),
                         (const float*)(din + o_th));
        if (rc) return rc;
        prof[9] += ns;
      }
      if (xdev()) {
        b.xr = ExRef();
        if (st.hsa() && (rc = publish(st, k % kIfStreams, nullptr, 0, &b.xr))) return rc;
      }
      if (int rc1 = lane_record(st, b.done)) return rc1;
      if (xdev() && g_shard_eager)
        if (int rc1 = exchange_start(b.d_x, b.done, b.xr, b.xbytes)) return rc1;
      tr(5, k, nl, maxN);
    }
    return EAO_OK;
  }
  // sharded: all-gather every rank's outcome of batch b, once, at its first
  // completion (no object of the batch has changed since the launch): per
  // owned object an outlier bit mask, then the owned speculative NP stats
  int exchange_batch(IfBatch& b) {
    const int nb = (int)b.objs.size();
    const size_t sb = sizeof(eao_np_stats);
    const size_t bytes = b.xbytes;
    const unsigned char* recv = nullptr;
    if (xdev()) {
      // the owner's kernels wrote the record into b.d_x; gathered on the GPU behind b.ev
      if (int rc = exchange_device(b.d_x, b.done, b.xr, bytes, &recv)) return rc;
    } else {
      if (b.launched) EAO_HIP_CHECK(spin_event(b.done));
      xsend.assign(bytes, 0);
      size_t w = 0;
      for (int c : b.lc) {
        const Obj* o = b.objs[c];
        const float th = o->cls == 62 ? 0.65f : 0.6f;
        const double* sc = (const double*)b.h_out + b.loff[c];
        const size_t n = o->pts.size();
        for (size_t k = 0; k < n; k++)
          if (sc[k] > th) xsend[w + k / 8] |= (unsigned char)(1u << (k % 8));
        w += (n + 7) / 8;
      }
      w = al16(w);  // the stats start 16-byte aligned (the device form stores them as structs)
      size_t j = 0;
      for (size_t q = 0; q < b.sp_obj.size(); q++)
        if (mine(b.objs[b.sp_obj[q]])) {  // launch order = sp_* order restricted to this rank
          std::memcpy(xsend.data() + w + sb * j, b.h_out + b.sp_out + sb * j, sb);
          j++;
        }
      if (int rc = exchange(bytes)) return rc;
      recv = xrecv.data();
    }
    const size_t stride = bytes;
    b.xres.assign(recv, recv + bytes * sworld);
    b.mask_off.assign(nb, 0);
    b.spst.resize(b.sp_obj.size());
    std::vector<size_t> cm(sworld, 0), cs(sworld, 0);
    for (int c = 0; c < nb; c++) {
      const int r = owner(b.objs[c]);
      b.mask_off[c] = stride * r + cm[r];
      cm[r] += (b.objs[c]->pts.size() + 7) / 8;
    }
    for (size_t q = 0; q < b.sp_obj.size(); q++) {
      const int r = owner(b.objs[b.sp_obj[q]]);
      std::memcpy(&b.spst[q], b.xres.data() + stride * r + al16(b.xmb[r]) + sb * cs[r]++, sb);
    }
    b.xdone = true;
    return EAO_OK;
  }
  int complete_forest(Obj* o) {
    if (!o->pending) return EAO_OK;
    if (o->slot < 0) {
      int rc = kick();
      if (rc) return rc;
      if (!o->pending) return EAO_OK;
    }
    Tick tk(&prof[3]);
    IfBatch& b = ifb[o->slot];
    if (!b.xdone) {
      int rc = exchange_batch(b);
      if (rc) return rc;
    } else if (b.launched) {
      Tick tw(&prof[39]);
      Tick tw2(&prof[42 + phase]);
      tr(6, o->slot, phase);
      // this object's scores and its speculative NP stats written (the batch's other objects
      // and kernels may still run) -- or the batch's event
      int c0 = 0;
      while (b.objs[c0] != o) c0++;
      const size_t s0 = (size_t)b.loff[c0], s1 = s0 + o->pts.size();
      size_t si = s0, qi = 0;
      const size_t nsw = sizeof(eao_np_stats) / 4;
      auto ready = [&]() -> bool {
        for (; si < s1; si++)
          if (ld64(b.h_out + 8 * si) == kSent64) return false;
        for (; qi < b.sp_obj.size(); qi++) {
          if (b.sp_obj[qi] != c0) continue;
          const unsigned char* st = b.h_out + b.sp_out + sizeof(eao_np_stats) * qi;  // unsharded: launch order
          for (size_t w = 0; w < nsw; w++)
            if (ld32(st + 4 * w) == kSent32) return false;
        }
        return true;
      };
      if (sharded()) {  // outputs come from the exchange; no sentinels there
        idle_work(b.done);
        EAO_HIP_CHECK(spin_event(b.done));
      } else {
        idle_work(b.done, ready);
        EAO_HIP_CHECK(spin_ready(b.done, ready));
        std::atomic_thread_fence(std::memory_order_acquire);
      }
      tr(7, o->slot, phase);
    }
    double tpost = now_us();
    int c = 0;
    while (b.objs[c] != o) c++;
    const size_t n = o->pts.size();
    size_t w = 0;
    if (sharded()) {
      const unsigned char* m = b.xres.data() + b.mask_off[c];
      for (size_t k = 0; k < n; k++) {
        if (m[k / 8] >> (k % 8) & 1) {
          for (int a = 0; a < 3; a++) o->sum[a] -= o->pts[k]->pos[a];
        } else {
          o->pts[w++] = o->pts[k];
        }
      }
    } else {
      const float th = o->cls == 62 ? 0.65f : 0.6f;
      const double* sc = (const double*)b.h_out + b.loff[c];
      for (size_t k = 0; k < n; k++) {
        if (sc[k] > th) {
          for (int a = 0; a < 3; a++) o->sum[a] -= o->pts[k]->pos[a];
        } else {
          o->pts[w++] = o->pts[k];
        }
      }
    }
    o->pts.resize(w);
    prof[40] += now_us() - tpost;
    if (o->pending == 2) mean_std(o);
    if (o->yaw_due) {  // SampleObjYaw of the launch frame, now that the cuboid is final
      o->yaw_due = false;
      sample_yaw(o, o->yawT);
    }
    const eao_np_stats* sps = sharded() ? b.spst.data() : (const eao_np_stats*)(b.h_out + b.sp_out);
    if (!o->dfr.empty()) {  // effects of later same-frame detections, in their order
      for (const Obj::Dfr& d : o->dfr) {
        if (d.kind == Obj::DFR_PROJ_IF_NP || d.kind == Obj::DFR_VOTE_IF_NP) {
          // NP verdict of (d.det, o) on the post-forest cloud: one of the speculative
          // pairs evaluated behind this forest (kick() includes every later detection)
          int v = -2;
          if (b.fid == d.det->fid)
            for (size_t q = 0; q < b.sp_obj.size(); q++)
              if (b.sp_obj[q] == c && b.sp_det[q] == d.det->index) {
                v = sps[q].verdict;
                break;
              }
          if (v < 0) {
            set_error(v == -2 ? "replay: deferred NP verdict missing" : "replay: NP pair outside kernel capacity");
            pend_err = v == -2 ? EAO_E_STATE : EAO_E_CAPACITY;
            continue;
          }
          if (v == 2) continue;  // fails: the object was not in vNP
        }
        if (d.kind == Obj::DFR_T) t_step_deferred(o, d);
        else if (d.kind == Obj::DFR_VOTE_IF_NP) reobj(d.target, o->id);
        else proj_with(o, o->dfrT);
      }
      o->dfr.clear();
      o->proj_dfr = false;
    }
    if (b.fid == cur)
      for (size_t q = 0; q < b.sp_obj.size(); q++)
        if (b.sp_obj[q] == c) np_cache[{b.sp_det[q], o->id}] = NpEntry{sps[q], b.sp_ver[q]};
    o->pending = 0;
    o->slot = -1;
    b.left--;
    return EAO_OK;
  }
  int flush(int cls) {
    for (auto& up : objs)
      if (up->pending && (cls < 0 || up->cls == cls)) {
        int rc = complete_forest(up.get());
        if (rc) return rc;
      }
    return EAO_OK;
  }
  // an object's points are about to be read: finish its forest first
  int touch(Obj* o) { return o->pending ? complete_forest(o) : EAO_OK; }
  int flush_list(const std::vector<Obj*>& todo) {
    for (Obj* o : todo) {
      int rc = touch(o);
      if (rc) return rc;
    }
    return EAO_OK;
  }

  void project_rect_host(Obj* o) {  // Object_Map::ComputeProjectRectFrame (one-off)
    if (touch(o)) return;
    if (o->pts.empty()) return;
    float xmn = INFINITY, xmx = -INFINITY, ymn = INFINITY, ymx = -INFINITY;
    for (MapPt* p : o->pts) {
      float u, v;
      proj_pt(p, u, v);
      xmn = std::min(xmn, u);
      xmx = std::max(xmx, u);
      ymn = std::min(ymn, v);
      ymx = std::max(ymx, v);
    }
    if (xmn < 0) xmn = 0;
    if (ymn < 0) ymn = 0;
    if (xmx > pz.cols) xmx = (float)pz.cols;
    if (ymx > pz.rows) ymx = (float)pz.rows;
    o->proj = rect_trunc(xmn, ymn, xmx - xmn, ymx - ymn);
  }

  // ComputeProjectRectFrame under a stored pose (a deferred recompute, complete_forest)
  void proj_with(Obj* o, const float* T) {
    if (o->pts.empty()) return;
    Pose pv = pz;
    std::memcpy(pv.T, T, sizeof(pv.T));
    float xmn = INFINITY, xmx = -INFINITY, ymn = INFINITY, ymx = -INFINITY;
    for (MapPt* p : o->pts) {
      float u, v;
      pv.proj(p->pos, u, v);
      xmn = std::min(xmn, u);
      xmx = std::max(xmx, u);
      ymn = std::min(ymn, v);
      ymx = std::max(ymx, v);
    }
    if (xmn < 0) xmn = 0;
    if (ymn < 0) ymn = 0;
    if (xmx > pz.cols) xmx = (float)pz.cols;
    if (ymx > pz.rows) ymx = (float)pz.rows;
    o->proj = rect_trunc(xmn, ymn, xmx - xmn, ymx - ymn);
  }
  void defer(Obj* o, const Obj::Dfr& d) {
    if (o->dfr.empty()) std::memcpy(o->dfrT, pz.T, sizeof(o->dfrT));
    o->dfr.push_back(d);
    if (d.kind != Obj::DFR_VOTE_IF_NP) o->proj_dfr = true;
  }
  void defer(Obj* o, int kind, Det* f, Obj* target) { defer(o, Obj::Dfr{kind, f, target}); }
  // the t-test step's rect part for a held object, at its forest's completion: the rect
  // read is the one the earlier deferred effects left (they are applied in order)
  void t_step_deferred(Obj* o, const Obj::Dfr& d) {
    const Det* f = d.det;
    int mem = 0;  // 1 vT, 2 vTL
    if (std::max(ov_iou(f->box, o->proj), ov_iou(f->feat, o->proj)) > 0.25) {
      mem = (d.t8 || d.m10) ? 1 : 2;
    } else if (d.m4) {
      proj_with(o, o->dfrT);  // ComputeProjectRectFrame under the detection's pose
      if (std::max(ov_iou(f->box, o->proj), ov_iou(f->feat, o->proj)) > 0.25) mem = 2;
    }
    if (!mem) return;
    if (d.mode == 1 && mem == 1) {
      proj_with(o, o->dfrT);  // DataAssociateUpdate(.., 3) of an updated object: the rect only
    } else if (d.target && d.target != o) {
      reobj(d.target, o->id);
    }
  }
  // an object updated earlier in this frame whose forest has not completed: a later
  // detection's decisions cannot associate it (DataAssociateUpdate returns false), so
  // its forest-dependent effects on them are deferred instead of waited for
  bool held(const Obj* o) const { return o->pending && o->last_add == (int)cur; }
  // o->proj is about to be read: apply a deferred recompute first
  int proj_read(Obj* o) { return o->proj_dfr ? touch(o) : EAO_OK; }

  // projected rects (step 10.1, Object_Map::ComputeProjectRectFrame) of `list`
  // and NoParaDataAssociation statistics of the (det, obj) `pairs`: one packed
  // upload of the points they read, two launches and one synchronisation.
  // Results: rects [5 per object: x, y, w, h, ok], stats [per pair].
  int rects_np_launch(const std::vector<Obj*>& list, const std::vector<std::pair<Det*, Obj*>>& pairs,
                      std::vector<int>& rects, std::vector<eao_np_stats>& stats) {
    const int nb = (int)list.size(), npairs = (int)pairs.size();
    rects.assign(5 * (size_t)nb, 0);
    stats.resize(npairs);
    if (nb == 0 && npairs == 0) return EAO_OK;
    std::unordered_map<const void*, int> offs;
    std::vector<const std::vector<MapPt*>*> srcs;  // point lists in upload order
    size_t total = 0;
    auto add = [&](const void* key, const std::vector<MapPt*>& v) {
      if (offs.emplace(key, (int)total).second) {
        srcs.push_back(&v);
        total += v.size();
      }
    };
    for (Obj* o : list) add(o, o->pts);
    for (auto& pr : pairs) {
      add(pr.first, pr.first->pts);
      add(pr.second, pr.second->pts);
    }
    // objects whose isolation forest is still running: their clouds are uploaded as they
    // stand and the kernels, queued behind the forest (event wait), drop the points the
    // forest erases on the fly -- the host completes the forest after this launch
    std::vector<const double*> os_l(nb, nullptr), os_p(npairs, nullptr);
    std::vector<float> th_l(nb, 0.f), th_p(npairs, 0.f);
    std::vector<int> wait_slots;
    bool chained = false;
    auto inflight = [&](Obj* o, const double*& ptr, float& th) {
      if (sharded() || !o->pending || o->slot < 0) return;
      IfBatch& b = ifb[o->slot];
      if (!b.launched) return;
      int c = 0;
      while (b.objs[c] != o) c++;
      ptr = (const double*)b.d_out + b.loff[c];
      th = o->cls == 62 ? 0.65f : 0.6f;
      chained = true;
      if (std::find(wait_slots.begin(), wait_slots.end(), o->slot) == wait_slots.end()) wait_slots.push_back(o->slot);
    };
    for (int b = 0; b < nb; b++) inflight(list[b], os_l[b], th_l[b]);
    for (int k = 0; k < npairs; k++) inflight(pairs[k].second, os_p[k], th_p[k]);
    // in: rect meta [2 nb] | pair meta [4 npairs] | Tcw [16] | points [3 total] | valid [total] |
    //     (chained) score pointers [nb + npairs] | thresholds [nb + npairs]
    // out: stats [npairs] | rects [4 nb] | ok [nb]
    const size_t o_pm = sizeof(int) * 2 * (size_t)nb, o_T = al16(o_pm + sizeof(int) * 4 * (size_t)npairs);
    const size_t o_pts = o_T + sizeof(float) * 16, o_val = o_pts + sizeof(float) * 3 * total;
    const size_t o_osp = al16(o_val + total), o_oth = o_osp + sizeof(double*) * (size_t)(nb + npairs);
    const size_t in_bytes = chained ? o_oth + sizeof(float) * (size_t)(nb + npairs) : o_val + total;
    const size_t o_r = sizeof(eao_np_stats) * (size_t)npairs, o_ok = o_r + sizeof(int) * 4 * (size_t)nb;
    // the previous frame start's wait may have ended on its outputs before its event: the event
    // is queried once before its pinned buffers are refilled, so a fault of that launch is
    // reported here (its outputs were complete: see spin_ready for the kernels' rules)
    if (gpu0.e || gpu0.sig) {
      const hipError_t e = done_query(gpu0);
      if (e != hipSuccess && e != hipErrorNotReady) EAO_HIP_CHECK(e);
    }
    int rc = stage(in_bytes, o_ok + nb);
    if (rc) return rc;
    if (int rc0 = lanes_init()) return rc0;
    // the packed inputs: pinned host memory the kernel reads in place, or (HSA lanes) device
    // memory written here through the BAR -- write-only (never read back on the host)
    unsigned char* hin = h_in;
    if (lanes_hsa && g_bar_fs) {
      if (in_bytes > cap_fs_bar) {
        // the previous frame start may still read the old buffer (see the forest batches)
        if (fs_bar && (gpu0.e || gpu0.sig)) EAO_HIP_CHECK(spin_event_plain(gpu0));
        const size_t c = std::max(in_bytes, 2 * cap_fs_bar);
        bar_free(fs_bar);
        cap_fs_bar = 0;
        fs_bar = (unsigned char*)bar_alloc(A->dev, c);
        if (fs_bar) cap_fs_bar = c;
      }
      if (fs_bar) hin = fs_bar;
    }
    // outputs: pinned host memory (read after the spin), or -- sharded, device-form
    // exchange -- this rank's record in device memory (d_out), all-gathered by the caller
    unsigned char* ob = rn_dev ? d_out : h_out;
    if (!rn_dev && g_sentinel) {  // outputs pre-filled with patterns the kernel never writes
      fill32(h_out, (size_t)npairs * (sizeof(eao_np_stats) / 4) + 4 * (size_t)nb);
      std::memset(h_out + o_ok, kSent8, (size_t)nb);
    }
    int* rmeta = (int*)hin;
    int* pmeta = (int*)(hin + o_pm);
    float* pts = (float*)(hin + o_pts);
    uint8_t* valid = hin + o_val;
    std::memcpy(hin + o_T, pz.T, sizeof(float) * 16);
    {
      Tick tpk(&prof[54]);
      prof[55] += (double)total;
      size_t o = 0;
      for (const std::vector<MapPt*>* v : srcs)
        for (MapPt* p : *v) {
          std::memcpy(&pts[3 * o], p->pos, sizeof(float) * 3);
          valid[o++] = p->bad ? 0 : 1;  // out_point is never set (Q7)
        }
    }
    for (int b = 0; b < nb; b++) {
      rmeta[b] = offs[list[b]];
      rmeta[nb + b] = (int)list[b]->pts.size();
    }
    int max_olen = 0;
    for (int k = 0; k < npairs; k++) {
      const auto& pr = pairs[k];
      const int olen = (int)pr.second->pts.size();
      pmeta[k] = offs[pr.first];
      pmeta[npairs + k] = (int)pr.first->pts.size();
      pmeta[2 * npairs + k] = offs[pr.second];
      pmeta[3 * npairs + k] = olen;
      if (olen > NP_MAXN && !os_p[k]) {  // chained: the kernel checks after the erasure
        set_error("replay: object exceeds the NP kernel capacity");
        return EAO_E_CAPACITY;
      }
      max_olen = std::max(max_olen, olen);
    }
    if (chained) {
      const double** osp = (const double**)(hin + o_osp);
      float* oth = (float*)(hin + o_oth);
      for (int b = 0; b < nb; b++) {
        osp[b] = os_l[b];
        oth[b] = th_l[b];
      }
      for (int k = 0; k < npairs; k++) {
        osp[nb + k] = os_p[k];
        oth[nb + k] = th_p[k];
      }
    }
    // queued behind the latest of those forests on its own stream when that batch is the
    // stream's last work (in-queue order: no cross-queue event wait on the chain, which
    // costs 10-25 us between the forest's end and this launch's start); the others, if
    // any, through event waits
    Lane ls = lanes_hsa ? fs_lane : Lane(A->stream);
    int lk = -1;
    for (int k : wait_slots)
      if (if_tail[k % kIfStreams] == k && (lk < 0 || ifb[k].seq > ifb[lk].seq)) lk = k;
    if (lk >= 0) {
      ls = if_stream[lk % kIfStreams];
      if_tail[lk % kIfStreams] = -1;
    }
    for (int k : wait_slots)
      if (k != lk)
        if (int rc0 = lane_wait(ls, ifb[k].done)) return rc0;
    // one launch reads the packed inputs in place (pinned host memory, or the BAR-written device
    // copy, flushed before the lane's doorbell) and writes the results straight back into pinned
    // host memory
    const unsigned char* din = hin;
    if (hin != h_in) lane_bar_written(ls, hin + in_bytes - 1);
    const int* drm = (const int*)din;
    const int* dpm = (const int*)(din + o_pm);
    const float* dpts = (const float*)(din + o_pts);
    const uint8_t* dval = din + o_val;
    const double* const* dosp = chained ? (const double* const*)(din + o_osp) : nullptr;
    const float* doth = chained ? (const float*)(din + o_oth) : nullptr;
    rc = A->rects_np(camdev, (const float*)(din + o_T), nb, dpts, drm, drm + nb, (int*)(ob + o_r), ob + o_ok,
                     dosp, doth, npairs, dpts, dval, dpm, dpm + npairs, dpts, dval, dpm + 2 * npairs, dpm + 3 * npairs,
                     (eao_np_stats*)ob, ls, max_olen, dosp ? dosp + nb : nullptr, doth ? doth + nb : nullptr);
    if (rc) return rc;
    fs_xr = ExRef();
    if (rn_dev && ls.hsa() && (rc = publish(ls, lane_index(ls), nullptr, 0, &fs_xr))) return rc;
    if (int rc0 = lane_record(ls, gpu0)) return rc0;
    tr(2, lk, (int)wait_slots.size(), npairs);
    if (phase == 0) {  // the frame start's launch: time since the frame began
      prof[58] += now_us() - frame_t0;
      prof[59] += 1;
    }
    if (rn_dev) return EAO_OK;
    {
      Tick tw(&prof[41]);
      // every stats word, every ok byte, and the rect words of the ok rects written (scanned
      // from where the last scan stopped)
      const size_t nsw = (size_t)npairs * (sizeof(eao_np_stats) / 4);
      size_t ws = 0;
      int wb = 0;
      auto ready = [&]() -> bool {
        for (; ws < nsw; ws++)
          if (ld32(h_out + 4 * ws) == kSent32) return false;
        for (; wb < nb; wb++) {
          const uint8_t okb = ld8(h_out + o_ok + wb);
          if (okb == kSent8) return false;
          if (okb)
            for (int q = 0; q < 4; q++)
              if (ld32(h_out + o_r + 4 * (4 * (size_t)wb + q)) == kSent32) return false;
        }
        return true;
      };
      idle_work(gpu0, ready);  // the next frame's steps 1-6, while the GPU is busy
      EAO_HIP_CHECK(spin_ready(gpu0, ready));
      std::atomic_thread_fence(std::memory_order_acquire);
    }
    tr(3);
    const int* r = (const int*)(h_out + o_r);
    const uint8_t* ok = h_out + o_ok;
    for (int b = 0; b < nb; b++) {
      for (int q = 0; q < 4; q++) rects[5 * b + q] = r[4 * b + q];
      rects[5 * b + 4] = ok[b];
    }
    if (npairs) std::memcpy(stats.data(), h_out, sizeof(eao_np_stats) * npairs);
    return EAO_OK;
  }

  // sharded form: each rank launches the objects (and pairs of objects) it
  // owns, then the records are all-gathered and re-assembled in list order
  int rects_np(const std::vector<Obj*>& list, const std::vector<std::pair<Det*, Obj*>>& pairs,
               std::vector<int>& rects, std::vector<eao_np_stats>& stats) {
    if (!sharded()) return rects_np_launch(list, pairs, rects, stats);
    for (auto& pr : pairs)  // capacity checked on every rank before the owner split (same verdict)
      if (pr.second->pts.size() > (size_t)NP_MAXN) {
        set_error("replay: object exceeds the NP kernel capacity");
        return EAO_E_CAPACITY;
      }
    std::vector<Obj*> L;
    std::vector<std::pair<Det*, Obj*>> P;
    std::vector<int> nl(sworld, 0), npr(sworld, 0);
    for (Obj* o : list) {
      nl[owner(o)]++;
      if (mine(o)) L.push_back(o);
    }
    for (auto& pr : pairs) {
      npr[owner(pr.second)]++;
      if (mine(pr.second)) P.push_back(pr);
    }
    std::vector<int> R;
    std::vector<eao_np_stats> S;
    const size_t sb = sizeof(eao_np_stats);
    if (xdev()) {
      // device form: the launch writes this rank's record [stats][rects x4][ok] into device
      // memory (rects_np_launch's own output layout); it is gathered there and only the
      // gathered records come back
      size_t bytes = 0;
      for (int q = 0; q < sworld; q++) bytes = std::max(bytes, sb * npr[q] + (sizeof(int) * 4 + 1) * nl[q]);
      bytes = std::max<size_t>(al16(bytes), 16);
      if (int rc = stage(0, bytes)) return rc;
      int rc;
      if (L.empty() && P.empty()) {  // nothing owned: an empty record
        if (int rc0 = lanes_init()) return rc0;
        fs_xr = ExRef();
        if (lanes_hsa) {
          if (int rc0 = publish(fs_lane, kIfStreams, d_out, bytes, &fs_xr)) return rc0;
          if (int rc0 = lane_record(fs_lane, gpu0)) return rc0;
        } else {
          EAO_HIP_CHECK(hipMemsetAsync(d_out, 0, bytes, A->stream));
          if (int rc0 = lane_record(Lane(A->stream), gpu0)) return rc0;
        }
      } else {
        rn_dev = true;
        rc = rects_np_launch(L, P, R, S);
        rn_dev = false;
        if (rc) return rc;
      }
      if (g_shard_eager && (rc = exchange_start(d_out, gpu0, fs_xr, bytes))) return rc;
      idle_work(gpu0);  // the next frame's steps 1-6, while the GPU is busy
      const unsigned char* recv = nullptr;
      if ((rc = exchange_device(d_out, gpu0, fs_xr, bytes, &recv))) return rc;
      std::vector<int> il(sworld, 0), ip(sworld, 0);
      rects.assign(5 * list.size(), 0);
      stats.resize(pairs.size());
      for (size_t b = 0; b < list.size(); b++) {
        const int q = owner(list[b]);
        const unsigned char* rec = recv + bytes * q;
        const int i = il[q]++;
        std::memcpy(&rects[5 * b], rec + sb * npr[q] + sizeof(int) * 4 * i, sizeof(int) * 4);
        rects[5 * b + 4] = rec[sb * npr[q] + sizeof(int) * 4 * nl[q] + i];
      }
      for (size_t k = 0; k < pairs.size(); k++) {
        const int q = owner(pairs[k].second);
        std::memcpy(&stats[k], recv + bytes * q + sb * ip[q]++, sb);
      }
      return EAO_OK;
    }
    int rc = rects_np_launch(L, P, R, S);
    if (rc) return rc;
    const size_t rb = sizeof(int) * 5;
    size_t bytes = 0;
    for (int q = 0; q < sworld; q++) bytes = std::max(bytes, rb * nl[q] + sb * npr[q]);
    xsend.assign(bytes, 0);
    if (!R.empty()) std::memcpy(xsend.data(), R.data(), rb * L.size());
    if (!S.empty()) std::memcpy(xsend.data() + rb * L.size(), S.data(), sb * P.size());
    if ((rc = exchange(bytes))) return rc;
    const size_t stride = xrecv.size() / sworld;
    std::vector<int> il(sworld, 0), ip(sworld, 0);
    rects.assign(5 * list.size(), 0);
    stats.resize(pairs.size());
    for (size_t b = 0; b < list.size(); b++) {
      const int q = owner(list[b]);
      std::memcpy(&rects[5 * b], xrecv.data() + stride * q + rb * il[q]++, rb);
    }
    for (size_t k = 0; k < pairs.size(); k++) {
      const int q = owner(pairs[k].second);
      std::memcpy(&stats[k], xrecv.data() + stride * q + rb * nl[q] + sb * ip[q]++, sb);
    }
    return EAO_OK;
  }

  // frame start: step 10.1 for the recent objects and the NP statistics of
  // every (kept detection, same-class object) pair, together
  int frame_start_gpu(const std::vector<Obj*>& list, const std::vector<std::pair<Det*, Obj*>>& pairs,
                      const std::vector<int>& di, const std::vector<int>& oi) {
    if (list.empty() && pairs.empty()) return EAO_OK;
    {
      Tick tfk(&prof[57]);
      if (int rc = kick()) return rc;  // pending forests overlap this launch
    }
    auto complete_pending = [&]() -> int {
      // forests left pending by the previous frame: their objects' points are read now
      Tick tk(&prof[17]);
      if (int rc = flush_list(list)) return rc;
      for (auto& pr : pairs)
        if (int rc = touch(pr.second)) return rc;
      return EAO_OK;
    };
    // one rank: the launch is queued behind those forests on the GPU (erasure applied on
    // the fly, rects_np_launch) and the host completes them afterwards, so the host never
    // waits twice; sharded, the forests complete first (their outcome is all-gathered)
    if (sharded())
      if (int rc = complete_pending()) return rc;
    std::vector<int> rects;
    std::vector<eao_np_stats> st;
    {
      Tick tk(&prof[7]);
      prof[6] += 1;
      if (int rc = rects_np(list, pairs, rects, st)) return rc;
    }
    // completion before the results are applied: a deferred projected-rect recompute of
    // the previous frame must not overwrite this frame's step 10.1 rect
    if (!sharded())
      if (int rc = complete_pending()) return rc;
    for (size_t b = 0; b < list.size(); b++)
      if (rects[5 * b + 4]) list[b]->proj = IRect(rects[5 * b], rects[5 * b + 1], rects[5 * b + 2], rects[5 * b + 3]);
    for (size_t k = 0; k < pairs.size(); k++) np_cache[{di[k], oi[k]}] = NpEntry{st[k], over[oi[k]]};
    return EAO_OK;
  }

  // NoParaDataAssociation statistics for the given (det, obj) pairs, one launch
  int np_pairs(const std::vector<std::pair<Det*, Obj*>>& pairs, const std::vector<int>& di,
               const std::vector<int>& oi) {
    if (pairs.empty()) return EAO_OK;
    if (int rc = kick()) return rc;  // pending forests overlap this launch
    Tick tk(&prof[5]);
    prof[4] += 1;
    std::vector<int> rects;
    std::vector<eao_np_stats> st;
    int rc = rects_np({}, pairs, rects, st);
    if (rc) return rc;
    for (size_t k = 0; k < pairs.size(); k++) np_cache[{di[k], oi[k]}] = NpEntry{st[k], over[oi[k]]};
    return EAO_OK;
  }

  int np_for_detection(Det* f) {
    std::vector<std::pair<Det*, Obj*>> pairs;
    std::vector<int> di, oi;
    for (size_t i = 0; i < objs.size(); i++) {
      Obj* o = objs[i].get();
      if (o->cls != f->cls || o->bad) continue;
      pairs.push_back({f, o});
      di.push_back(f->index);
      oi.push_back((int)i);
    }
    return np_pairs(pairs, di, oi);
  }

  static void vote(MapPt* p, int id) {
    int* v = p->vote_of(id);
    if (v) *v += 1;
    else p->votes.push_back({id, 1});
  }
  static void reobj(Obj* o, int id) {
    auto it = o->reobj.find(id);
    if (it != o->reobj.end()) it->second += 1;
    else o->reobj[id] = 1;
  }

  void mark_dirty(Obj* o) {
    if ((size_t)o->id >= over.size()) over.resize(o->id + 1, 0);
    over[o->id]++;
  }
  bool np_fresh(int det, int i) const {
    auto it = np_cache.find({det, i});
    return it != np_cache.end() && (size_t)i < over.size() && it->second.ver == over[i];
  }

  // Object_Map::DataAssociateUpdate, Object.cc:1313-1554
  bool update(Obj* o, Det* f, int Flag) {
    Tick tku(&prof[28]);
    if (f->cls != o->cls) return false;
    if (held(o)) {
      // already updated in this frame: the reference returns false at the mnLastAddID
      // check below; of the work before it only the projected rect of flags 2/3 (from the
      // post-forest points) is an effect, and it is deferred to the forest's completion
      if (Flag == 2 || Flag == 3) defer(o, Obj::DFR_PROJ, f, nullptr);
      return false;
    }
    phase = 9;
    if (touch(o)) return false;
    phase = 1;
    if (Flag != 1 && Flag != 4) {
      project_rect_host(o);
      const IRect r1 = o->proj;
      float xmn = INFINITY, xmx = -INFINITY, ymn = INFINITY, ymx = -INFINITY;
      auto acc = [&](MapPt* p) {
        float u, v;
        proj_pt(p, u, v);
        xmn = std::min(xmn, u);
        xmx = std::max(xmx, u);
        ymn = std::min(ymn, v);
        ymx = std::max(ymx, v);
      };
      for (MapPt* p : f->pts) acc(p);
      for (MapPt* p : o->pts) acc(p);
      if (xmn < 0) xmn = 0;
      if (ymn < 0) ymn = 0;
      if (xmx > pz.cols) xmx = (float)pz.cols;
      if (ymx > pz.rows) ymx = (float)pz.rows;
      const IRect r2 = rect_trunc(xmn, ymn, xmx - xmn, ymx - ymn);
      if ((ov_iou(r1, r2) < 0.5) && (ov_former(r2, f->box) < 0.8)) return false;
    }
    if (o->last_add != (int)cur) {
      o->lastlast_add = o->last_add;
      o->last_add = (int)cur;
      o->lastlast = o->last;
      o->last = f->box;
      o->conf++;
      o->frames.push_back(f);
    } else
      return false;
    mark_dirty(o);
    f->mnId = o->id;
    double qi[4], ti[3];  // cuboid pose inverse, the same for every point
    se3_inverse(o->q, o->t, qi, ti);
    PosSet& have = posset;
    have.reset(o->pts.size() + f->pts.size());
    for (MapPt* q : o->pts) {
      PosKey k;
      if (pos_key(q->pos, k)) have.insert(k);
    }
    for (MapPt* p : f->pts) {
      float d[3];
      for (int a = 0; a < 3; a++) d[a] = o->center[a] - p->pos[a];
      const float fDis = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
      const float th = o->frames.size() > 5 ? 0.9f : 1.0f;
      if (fDis > th * o->rmax) continue;
      if (o->frames.size() >= 10 && (o->cls == 56 || o->cls == 77)) {
        const double v[3] = {p->pos[0], p->pos[1], p->pos[2]};
        double s[3];
        se3_apply(qi, ti, v, s);
        if (std::fabs(s[0]) > 1.2 * o->lenth / 2 || std::fabs(s[1]) > 1.2 * o->width / 2 ||
            std::fabs(s[2]) > 1.2 * o->height / 2)
          continue;
      }
      vote(p, o->id);
      PosKey k;
      const bool finite = pos_key(p->pos, k);
      if (!finite || !have.contains(k)) {
        o->pts.push_back(p);
        for (int a = 0; a < 3; a++) o->sum[a] += p->pos[a];
        if (finite) have.insert(k);
      }
    }
    if (f->bx > 25 && f->by > 25 && f->bx + f->bw < pz.cols - 25 && f->by + f->bh < pz.rows - 25) {
      size_t w = 0;
      const size_t n = o->pts.size();
      for (size_t i = 0; i < n; i++) {
        MapPt* p = o->pts[i];
        const int* vp = p->vote_of(o->id);
        const int votes = vp ? *vp : 0;
        bool erase = false;
        if (votes <= 8) {
          float u, v;
          proj_pt(p, u, v);
          if ((u > 0 && u < pz.cols) && (v > 0 && v < pz.rows) && !f->box.contains_f(u, v)) erase = true;
        }
        if (erase) {
          for (int a = 0; a < 3; a++) o->sum[a] -= p->pos[a];
        } else {
          o->pts[w++] = p;
        }
      }
      o->pts.resize(w);
    }
    mean_std(o);
    o->pending = std::max(o->pending, 1);  // isolation forest: batched launch, applied on next read
    return true;
  }

  // Object_2D::ObjectDataAssociation, Object.cc:162-710
  int associate(Det* f) {
    if (flag == "None") biForest = false;
    cur_np_done = false;
    int rc;
    {
      Tick tk(&prof[16]);
      // same-class objects with a pending forest were updated earlier in this frame (the
      // frame start completed the older ones): they are held, not waited for (held());
      // launch their forests now, with this and every later detection's NP pairs behind them
      bool launch = false;  // a held same-class object whose forest is not in flight yet
      for (auto& up : objs)
        if (up->cls == f->cls && up->pending) {
          if (!held(up.get())) {
            phase = 5;
            if ((rc = touch(up.get()))) return rc;
            phase = 1;
          } else if (up->slot < 0) {
            launch = true;
          }
        }
      // launch it now (with this detection's NP pair behind it); objects of other classes
      // keep accumulating into the next batch (fewer, larger launches)
      rc = launch ? kick() : EAO_OK;
    }
    if (rc) return rc;
    const IRect RC = f->box;
    float IouMax = 0;
    bool byIou = false;
    int iouId = -1, iouMax = -1;
    float IouThreshold = 0.5;
    if (flag != "NA" && flag != "NP") {
      for (int i = 0; i < (int)objs.size(); i++) {
        Obj* o = objs[i].get();
        if (f->cls != o->cls || o->bad) continue;
        if ((unsigned long)(long)o->last_add == cur - 1) {
          IRect RP;
          if ((unsigned long)(long)o->lastlast_add == cur - 2) {
            float ltx = (float)(o->last.x * 2 - o->lastlast.x);
            if (ltx < 0) ltx = 0;
            float lty = (float)(o->last.y * 2 - o->lastlast.y);
            if (lty < 0) lty = 0;
            float rdx = (float)((o->last.x + o->last.w) * 2 - (o->lastlast.x + o->lastlast.w));
            if (ltx > pz.cols) rdx = (float)pz.cols;
            float rdy = (float)((o->last.y + o->last.h) * 2 - (o->lastlast.y + o->lastlast.h));
            if (lty > pz.rows) rdy = (float)pz.rows;
            RP = rect_trunc(ltx, lty, rdx - ltx, rdy - lty);
            IouThreshold = 0.6f;
          } else
            RP = o->last;
          const float I = ov_iou(RC, RP);
          if ((I > IouThreshold) && I > IouMax) {
            IouMax = I;
            iouMax = i;
          }
        }
      }
      if (IouMax > 0 && iouMax >= 0 && update(objs[iouMax].get(), f, 1)) {
        byIou = true;
        iouId = iouMax;
        f->method = 1;
      }
    }
    bool byNp = false;
    int npId = -1;
    std::vector<int> vNP;
    if (flag != "NA" && flag != "IoU") {
      // m counts valid frame points (bad ones were dropped in ComputeMeanAndStandardFrame;
      // out_point is never set, Q7). m < 20 breaks the loop at its first object (Q9).
      const bool m_small = f->pts.size() < 20;
      std::vector<int> need;
      if (!m_small) {
        for (int i = (int)objs.size() - 1; i >= 0; i--) {
          Obj* o = objs[i].get();
          if (f->cls != o->cls || o->bad) continue;
          if (byIou && i == iouId) continue;  // its verdict is never used (Object.cc:283-284)
          if (held(o)) continue;  // verdict at its forest's completion
          if (!np_fresh(f->index, i)) need.push_back(i);
        }
      }
      if (!need.empty()) {
        std::vector<Obj*> tl;
        for (int i : need) tl.push_back(objs[i].get());
        phase = 6;
        rc = flush_list(tl);  // completing a forest publishes its speculative NP pairs
        phase = 1;
        if (rc) return rc;
        std::vector<int> still;
        for (int i : need)
          if (!np_fresh(f->index, i)) still.push_back(i);
        need.swap(still);
      }
      if (!need.empty()) {
        std::vector<std::pair<Det*, Obj*>> pairs;
        std::vector<int> di;
        for (int i : need) {
          pairs.push_back({f, objs[i].get()});
          di.push_back(f->index);
        }
        rc = np_pairs(pairs, di, need);
        if (rc) return rc;
      }
      cur_np_done = true;
      // vNP in the reference's order; a held object (verdict pending) enters as -1 - i:
      // it would fail DataAssociateUpdate, so it only decides votes and a rect recompute
      std::vector<int> ord;
      for (int i = (int)objs.size() - 1; i >= 0; i--) {
        Obj* o = objs[i].get();
        if (f->cls != o->cls || o->bad) continue;
        if (m_small) break;  // verdict 0
        if (byIou && i == iouId) continue;
        if (held(o)) {
          ord.push_back(-1 - i);
          continue;
        }
        const int v = np_cache[{f->index, i}].st.verdict;
        if (v < 0) {
          set_error("replay: NP pair outside kernel capacity");
          return EAO_E_CAPACITY;
        }
        if (v == 2) continue;
        vNP.push_back(i);
        ord.push_back(i);
      }
      if (byIou) {
        for (int k : ord) {
          if (k >= 0) {
            if (k != iouId) reobj(objs[iouId].get(), objs[k]->id);
          } else {
            defer(objs[-1 - k].get(), Obj::DFR_VOTE_IF_NP, f, objs[iouId].get());
          }
        }
      } else {
        Obj* won = nullptr;
        for (int k : ord) {
          if (!won) {
            if (k < 0) {
              // in vNP iff it passes: its failed update would recompute its projected rect
              defer(objs[-1 - k].get(), Obj::DFR_PROJ_IF_NP, f, nullptr);
            } else if (update(objs[k].get(), f, 2)) {
              byNp = true;
              npId = k;
              f->method = 2;
              won = objs[k].get();
            }
          } else if (k >= 0) {
            reobj(won, objs[k]->id);
          } else {
            defer(objs[-1 - k].get(), Obj::DFR_VOTE_IF_NP, f, won);
          }
        }
      }
    }
    bool byPro = false;
    int proId = -1;
    std::vector<int> vPro;
    if (flag != "NA" && flag != "IoU" && flag != "NP") {
      float fmax = 0.0f;
      int pmax = -1;
      for (int i = (int)objs.size() - 1; i >= 0; i--) {
        Obj* o = objs[i].get();
        if (f->cls != o->cls || o->bad) continue;
        if (f->pts.size() >= 10 && (int)o->frames.size() > 8) continue;
        phase = 7;
        if ((rc = proj_read(o))) return rc;
        phase = 1;
        const float a = std::max(ov_iou(RC, o->proj), ov_iou(f->feat, o->proj));
        if (a >= 0.25 && a > fmax) {
          fmax = a;
          pmax = i;
          vPro.push_back(i);
        }
      }
      if (fmax >= 0.25) {
        std::sort(vPro.begin(), vPro.end());
        if (byIou || byNp) {
          for (int j = (int)vPro.size() - 1; j >= 0; j--) {
            int re = -1;
            if (byIou) re = iouId;
            if (byNp) re = npId;
            if (vPro[j] != re) reobj(objs[re].get(), objs[vPro[j]]->id);
          }
        } else {
          if (update(objs[pmax].get(), f, 4)) {
            byPro = true;
            proId = pmax;
            f->method = 4;
          }
          for (int j = (int)vPro.size() - 1; j >= 0; j--)
            if (vPro[j] != pmax) reobj(objs[pmax].get(), objs[vPro[j]]->id);
        }
      }
    }
    bool byT = false;
    std::vector<int> vT, vTL;
    std::vector<std::pair<int, Obj::Dfr>> tdef;  // held objects' deferred t-test parts
    if (flag != "NA" && flag != "IoU" && flag != "NP") {
      for (int i = (int)objs.size() - 1; i >= 0; i--) {
        Obj* o = objs[i].get();
        if (f->cls != o->cls || o->bad) continue;
        const int df = (int)o->frames.size();
        if (df <= 8) continue;
        if (o->pending == 2 && (rc = proj_read(o))) return rc;  // completion recomputes center / csd
        const float dx = std::fabs(o->center[0] - f->pos[0]), dy = std::fabs(o->center[1] - f->pos[1]),
                    dz = std::fabs(o->center[2] - f->pos[2]);
        const float tx = (float)(dx / (o->csd[0] / std::sqrt((double)df)));
        const float ty = (float)(dy / (o->csd[1] / std::sqrt((double)df)));
        const float tz = (float)(dz / (o->csd[2] / std::sqrt((double)df)));
        const float* row = kTTable[std::min(df - 1, 121)];
        if (tx < row[5] && ty < row[5] && tz < row[5]) {
          vT.push_back(i);
          continue;
        }
        if (held(o) && o->pending == 1) {
          // the rect overlap decides from here on and reads the post-forest rect: a held
          // object cannot win the step (its update fails), so its part is deferred
          const Obj::Dfr d{Obj::DFR_T, f, nullptr, 0, (uint8_t)(tx < row[8] && ty < row[8] && tz < row[8]),
                           (uint8_t)((tx + ty + tz) / 3 < 10), (uint8_t)((tx + ty + tz) / 3 < 4)};
          tdef.push_back({i, d});
          continue;
        }
        phase = 8;
        if ((rc = proj_read(o))) return rc;
        phase = 1;
        const float a = std::max(ov_iou(RC, o->proj), ov_iou(f->feat, o->proj));
        if (a > 0.25) {
          if (tx < row[8] && ty < row[8] && tz < row[8])
            vT.push_back(i);
          else if ((a > 0.25) && ((tx + ty + tz) / 3 < 10))
            vT.push_back(i);
          else
            vTL.push_back(i);
        } else if ((tx + ty + tz) / 3 < 4) {
          project_rect_host(o);
          if (std::max(ov_iou(RC, o->proj), ov_iou(f->feat, o->proj)) > 0.25) vTL.push_back(i);
        }
      }
      if (byIou || byNp || byPro) {
        int re = -1;
        if (byIou) re = iouId;
        if (byNp) re = npId;
        if (byPro) re = proId;
        for (int k : vT)
          if (k != re) reobj(objs[re].get(), objs[k]->id);
        for (int k : vTL)
          if (k != re) reobj(objs[re].get(), objs[k]->id);
        for (auto& td : tdef) {
          td.second.target = objs[re].get();
          defer(objs[td.first].get(), td.second);
        }
      } else {
        int won = -1;  // objs index of the winner
        for (size_t i = 0; i < vT.size(); i++) {
          if (update(objs[vT[i]].get(), f, 3)) {
            byT = true;
            won = vT[i];
            const int tid = vT[i];
            f->method = 3;
            for (size_t j = i + 1; j < vT.size(); j++) reobj(objs[tid].get(), objs[vT[j]]->id);
            for (int k : vTL)
              if (k != tid) reobj(objs[tid].get(), objs[k]->id);
            break;
          }
        }
        for (auto& td : tdef) {  // vT runs in descending index: before the winner = above it
          td.second.mode = (won < 0 || td.first > won) ? 1 : 2;
          td.second.target = won >= 0 ? objs[won].get() : nullptr;
          defer(objs[td.first].get(), td.second);
        }
      }
    }
    if (byIou || byNp || byPro || byT) return EAO_OK;
    if (f->bx < 10 || f->by < 10 || f->bx + f->bw > pz.cols - 10 || f->by + f->bh > pz.rows - 10) {
      f->bad = true;
      return EAO_OK;
    }
    std::unique_ptr<Obj> o(new Obj());
    o->frames.push_back(f);
    o->id = (int)objs.size();
    o->cls = f->cls;
    o->conf = 1;
    o->last_add = o->lastlast_add = (int)cur;
    o->last = f->box;
    for (int a = 0; a < 3; a++) {
      o->sum[a] = f->sum[a];
      o->center[a] = f->pos[a];
    }
    for (MapPt* p : f->pts) {
      p->vote_insert(o->id, 1);
      o->pts.push_back(p);
    }
    f->mnId = o->id;
    f->method = 5;
    f->alias = o.get();
    o->pending = 2;  // IsolationForestDeleteOutliers then ComputeMeanAndStandard
    Obj* op = o.get();
    objs.push_back(std::move(o));
    mark_dirty(op);
    return EAO_OK;
  }

  void frame_mean(Det* f) {  // Object_2D::ComputeMeanAndStandardFrame, Object.cc:63-102
    size_t w = 0;
    for (size_t i = 0; i < f->pts.size(); i++) {
      MapPt* p = f->pts[i];
      if (p->bad) {
        for (int a = 0; a < 3; a++) f->sum[a] -= p->pos[a];
      } else
        f->pts[w++] = p;
    }
    f->pts.resize(w);
    const float sc = (float)(1. / (double)f->pts.size());
    for (int a = 0; a < 3; a++) f->pos[a] = f->sum[a] * sc + 0.0f;
  }

  void boxplot(Det* f, const Pose& P) {  // Object_2D::RemoveOutliersByBoxPlot, Object.cc:106-158
    std::vector<float> zc(f->pts.size());
    for (size_t i = 0; i < f->pts.size(); i++) {
      float pc[3];
      P.cam(f->pts[i]->pos, pc);
      zc[i] = pc[2];
    }
    std::vector<float> zs = zc;
    std::sort(zs.begin(), zs.end());
    if ((zs.size() / 4 <= 0) || (zs.size() * 3 / 4 >= zs.size() - 1)) return;
    const float Q1 = zs[zs.size() / 4], Q3 = zs[zs.size() * 3 / 4];
    const float IQR = Q3 - Q1;
    const float max_th = (float)(Q3 + 1.5 * IQR);
    size_t w = 0;
    for (size_t i = 0; i < f->pts.size(); i++)
      if (!(zc[i] > max_th)) f->pts[w++] = f->pts[i];
    f->pts.resize(w);
    frame_mean(f);
  }

  // LocalMapping's map-point changes (LocalBundleAdjustment SetWorldPos, MapPointCulling /
  // KeyFrameCulling SetBadFlag, SearchInNeighbors Replace; LocalMapping.cc:60-80,
  // MapPoint.cc:73-77,151-220) for the points the replay knows. The object code reads
  // GetWorldPos() / isBad() live at every later read (Object.cc:967-992), so the arena copy
  // is rewritten. Replace(pMP) leaves the object holding the old, now bad, pointer -- no
  // membership moves -- so it arrives here as a bad flag.
  int update_points(int n, const int32_t* ids, const float* pos, const uint8_t* bad) {
    // a pending forest's completion (ComputeMeanAndStandard of a new object, deferred
    // effects) must read the state the reference read when it ran the update: finish
    // the pending forests before the first change of a known point
    bool pend = false;
    for (auto& up : objs) pend |= up->pending != 0;
    for (int i = 0; pend && i < n; i++) {
      const MapPt* p = mp_lookup(ids[i]);
      if (!p) continue;
      if ((pos && std::memcmp(p->pos, pos + 3 * (size_t)i, sizeof(float) * 3) != 0) ||
          (bad && p->bad != (bad[i] != 0))) {
        if (int rc = flush(-1)) return rc;
        pend = false;
      }
    }
    for (int i = 0; i < n; i++) {
      MapPt* p = mp_lookup(ids[i]);
      if (!p) continue;  // never tracked: nothing holds it
      if ((pos && std::memcmp(p->pos, pos + 3 * (size_t)i, sizeof(float) * 3) != 0) ||
          (bad && p->bad != (bad[i] != 0)))
        point_changed(p);
      if (pos) {
        std::memcpy(p->pos, pos + 3 * (size_t)i, sizeof(float) * 3);
        p->proj_epoch = 0;
      }
      if (bad) p->bad = bad[i] != 0;
    }
    return EAO_OK;
  }
  // ids of the map points the objects hold (ascending, unique): what a LocalMapping shim
  // snapshots after BA / culling / fuse
  int held_points(std::vector<int32_t>& out) const {
    out.clear();
    for (const auto& up : objs)
      for (const MapPt* p : up->pts) out.push_back(p->id);
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
    return (int)out.size();
  }

  bool overlap(Obj* a, Obj* b) {  // Object_Map::WhetherOverlap, Object.cc:1906-1922
    const float dx = (float)std::fabs(a->center_c[0] - b->center_c[0]);
    const float dy = (float)std::fabs(a->center_c[1] - b->center_c[1]);
    const float dz = (float)std::fabs(a->center_c[2] - b->center_c[2]);
    return dx < a->lenth / 2 + b->lenth / 2 && dy < a->width / 2 + b->width / 2 &&
           dz < a->height / 2 + b->height / 2;
  }

  // ---- look-ahead (eao_replay_run): steps 1-6 of the next frame -- the frame's own points,
  // boxes and lines, independent of this frame's association -- run while this frame waits on
  // the GPU. Only when the next frame leaves every known map point's position and flag as they
  // stand (so nothing this frame's pending work reads changes), no map-point record comes in
  // between and the object map is initialised (no InitObjMap in step 9).
  struct FrameIn {
    unsigned long fid = 0;
    const float* T = nullptr;
    int nb = 0, npts = 0;
    const int32_t *boxes = nullptr, *ids = nullptr;
    const float *pos = nullptr, *uv = nullptr;
    const uint8_t* bad = nullptr;
  };
  FrameIn la;            // the next frame's inputs (set by the stream call)
  bool la_set = false;
  // steps 1-6 of one frame as a resumable sequence of short steps (a few us each), so idle
  // time is filled without holding the host past the GPU result it waits for
  struct Prep {
    bool active = false;  // being prepared ahead (look-ahead)
    bool ok = false;      // ... and complete
    FrameIn in;
    Pose P;
    int phase = 0;
    size_t k = 0;
    std::vector<MapPt*> tr;
    std::vector<Det*> o2, kept;
    bool took_lines = false;  // step 3 consumed a staged line set (staged_next moved past it)
    std::vector<int> created;  // map-point ids step 1 created (look-ahead only: erased on discard)
  } prep, prep_now;
  // drop a look-ahead that will not be consumed (a failed stream call, or a frame call that
  // does not continue the stream): its detections stay unreferenced, a line set it consumed
  // goes back to the front of the staged sets, and the frame runs in order when it comes
  // (the map points it created go too: a caller that resumes with another frame must not find
  // them among the known points, e.g. in eao_replay_update_points)
  void discard_lookahead() {
    if (prep.active && prep.took_lines && staged_next > 0) staged_next--;  // the set is still staged
    if (prep.active)
      for (int id : prep.created) mp_erase(id);
    prep.active = prep.ok = prep.took_lines = false;
    prep.o2.clear();
    prep.kept.clear();
    prep.created.clear();
    la_set = false;
  }
  // fill a wait on `ev` with the next frame's steps 1-6 (until the event, or `ready()`)
  void idle_work(const Done& ev) {
    idle_work(ev, [] { return false; }, false);
  }
  // (with a sentinel test the cheap ready() runs after every step and hipEventQuery, a runtime
  // call, after every fourth)
  template <class Ready>
  void idle_work(const Done& ev, Ready&& ready, bool has_ready = true) {
    if (!prep.active) {
      if (!g_lookahead || !la_set || prep.ok || !ini) return;
      la_set = false;
      for (int i = 0; i < la.npts; i++) {
        const MapPt* p = mp_lookup(la.ids[i]);
        if (!p) continue;
        if (std::memcmp(p->pos, la.pos + 3 * (size_t)i, sizeof(float) * 3) != 0 ||
            p->bad != (la.bad ? la.bad[i] != 0 : false))
          return;  // the next frame changes a known point: it runs in order
      }
      prep_begin(prep, la);
      std::memcpy(prep.P.T, la.T, sizeof(prep.P.T));
      prep.active = true;
      prof[53] += 1;
    }
    Tick tk(&prof[52]);
    const unsigned qmask = (g_sentinel && has_ready) ? 3u : 0u;
    for (unsigned it = 0; !prep.ok; it++) {
      if (g_la_eager) {
        prep.ok = prep_step(prep);
        continue;
      }
      if (g_sentinel && has_ready && ready()) break;
      if ((it & qmask) == 0 && done_query(ev) != hipErrorNotReady) break;
      prep.ok = prep_step(prep);
    }
  }
  void prep_begin(Prep& s, const FrameIn& in) {
    s.in = in;
    s.P = pz;
    s.phase = 0;
    s.k = 0;
    s.ok = false;
    s.took_lines = false;
    s.o2.clear();
    s.kept.clear();
    s.created.clear();
  }

  // STEPS 1-6 of TrackWithMotionModel's object section for one frame's inputs (pose s.P),
  // one bounded step per call; true when the frame is ready for step 9 / 10
  bool prep_step(Prep& s) {
    const FrameIn& in = s.in;
    const Pose& P = s.P;
    std::vector<Det*>& o2 = s.o2;
    const double tA = now_us();
    switch (s.phase) {
      case 0: {
        for (int k = 0; k < in.nb; k++) {
          std::unique_ptr<Det> f(new Det());
          f->cls = in.boxes[5 * k];
          f->bx = in.boxes[5 * k + 1];
          f->by = in.boxes[5 * k + 2];
          f->bw = in.boxes[5 * k + 3];
          f->bh = in.boxes[5 * k + 4];
          f->box = IRect(f->bx, f->by, f->bw, f->bh);
          f->index = k;
          f->fid = in.fid;
          o2.push_back(f.get());
          dets.push_back(std::move(f));
        }
        s.tr.resize(in.npts);
        s.phase = 1;
        s.k = 0;
        prof[12] += now_us() - tA;
        return false;
      }
      case 1: {  // the frame's map points, kPrepChunk per step
        const int e = std::min(in.npts, (int)s.k + kPrepChunk);
        const bool ahead = &s == &prep;
        for (int i = (int)s.k; i < e; i++) {
          if (ahead && !mp_lookup(in.ids[i])) s.created.push_back(in.ids[i]);
          MapPt* p = mappoint(in.ids[i]);
          const bool nb = in.bad ? in.bad[i] != 0 : false;
          if (std::memcmp(p->pos, in.pos + 3 * (size_t)i, sizeof(float) * 3) != 0 || p->bad != nb) point_changed(p);
          for (int a = 0; a < 3; a++) p->pos[a] = in.pos[3 * i + a];
          p->proj_epoch = 0;
          p->bad = nb;
          s.tr[i] = p;
        }
        s.k = (size_t)e;
        if (e >= in.npts) {
          s.phase = 2;
          s.k = 0;
        }
        prof[12] += now_us() - tA;
        return false;
      }
      case 2: {  // STEP 2 AssociateObjAndPoints, Tracking.cc:2434-2468 (in point order, kPrepChunk per step)
        const float* uv = in.uv;
        const int e = std::min(in.npts, (int)s.k + kPrepChunk);
        for (int i = (int)s.k; i < e; i++) {
          MapPt* p = s.tr[i];
          if (p->bad) continue;
          const int px = (int)lrintf(uv[2 * i]), py = (int)lrintf(uv[2 * i + 1]);
          for (Det* f : o2)
            if (f->box.contains_i(px, py)) {
              p->fu = uv[2 * i];
              p->fv = uv[2 * i + 1];
              f->pts.push_back(p);
              for (int a = 0; a < 3; a++) f->sum[a] += p->pos[a];
            }
        }
        s.k = (size_t)e;
        if (e >= in.npts) s.phase = 3;
        prof[12] += now_us() - tA;
        return false;
      }
      case 3:
        // STEP 3, Tracking.cc:1286 (a split frame takes its lines at eao_replay_frame_end: their only
        // reader is SampleObjYaw, at step 10.6 and at forest completions of later frames)
        if (!defer_lines || &s == &prep) associate_lines(o2, &s == &prep ? &s.took_lines : nullptr);
        s.phase = 4;
        s.k = 0;
        prof[12] += now_us() - tA;
        return false;
      case 4:  // STEP 4, one detection per step
        if (s.k < o2.size()) {
          Det* f = o2[s.k++];
          frame_mean(f);
          if (f->pts.size() >= 8) boxplot(f, P);
        }
        if (s.k >= o2.size()) s.phase = 5;
        prof[13] += now_us() - tA;
        return false;
      default:
        break;
    }
    for (Det* f : o2) {  // STEP 5
      const float sc = (float)(1. / (double)f->pts.size());
      for (int a = 0; a < 3; a++) f->pos[a] = f->sum[a] * sc + 0.0f;
      if (f->pts.size() < 4) continue;
      float xmn = INFINITY, xmx = -INFINITY, ymn = INFINITY, ymx = -INFINITY;
      for (MapPt* p : f->pts) {
        xmn = std::min(xmn, p->fu);
        xmx = std::max(xmx, p->fu);
        ymn = std::min(ymn, p->fv);
        ymx = std::max(ymx, p->fv);
      }
      if (xmn < 0) xmn = 0;
      if (ymn < 0) ymn = 0;
      if (xmx > P.cols) xmx = (float)P.cols;
      if (ymx > P.rows) ymx = (float)P.rows;
      f->feat = rect_trunc(xmn, ymn, xmx - xmn, ymx - ymn);
    }
    // STEP 6 filters, Tracking.cc:1383-1487
    for (size_t a = 0; a < o2.size(); a++) {
      int num = 0;
      for (size_t b = 0; b < o2.size(); b++)
        if (a != b && ov_latter(o2[a]->box, o2[b]->box) > 0.05) num++;
      if (num > 4) o2[a]->bad = true;
    }
    for (size_t a = 0; a < o2.size(); a++) {
      Det* f = o2[a];
      if (f->bad) continue;
      if (f->cls == 0 || f->cls == 63 || f->cls == 15) f->bad = true;
      if ((float)f->box.area() / (float)(P.cols * P.rows) > 0.5) f->bad = true;
      if (f->pts.size() < 5)
        f->bad = true;
      else if (f->pts.size() < 10 &&
               (f->bx < 20 || f->by < 20 || f->bx + f->bw > P.cols - 20 || f->by + f->bh > P.rows - 20))
        f->bad = true;
      for (size_t b = 0; b < o2.size(); b++) {
        Det* g = o2[b];
        if (g->bad || a == b) continue;
        if (ov_iou(f->box, g->box) > 0.3) {
          if (f->score < g->score) f->bad = true;
          else if (f->score >= g->score) g->bad = true;
        }
        if (ov_iou(f->box, g->box) > 0.05) {
          if (ov_former(f->box, g->box) > 0.85) f->bad = true;
          if (ov_latter(f->box, g->box) > 0.85) g->bad = true;
        }
      }
    }
    for (Det* f : o2) {
      if (!f->bad) s.kept.push_back(f);
      else f->method = -1;
    }
    prof[13] += now_us() - tA;
    return true;
  }

  // a frame split at its lines (eao_replay_frame_begin / _end): what the tail needs
  bool defer_lines = false;
  struct {
    bool open = false, step10 = false;
    unsigned long fid = 0;
    std::vector<Det*> o2;
  } split;
  int frame(unsigned long fid, const float* Tcw, int nb, const int32_t* boxes, int npts,
            const int32_t* ids, const float* pos, const float* uv, const uint8_t* bad, int32_t* out,
            bool begin_only = false) {
    if (split.open) return EAO_E_STATE;
    defer_lines = begin_only;
    struct DeferOff {
      bool* f;
      ~DeferOff() { *f = false; }
    } defer_off{&defer_lines};
    bool step10 = false;
    int rc0 = frame_body(fid, Tcw, nb, boxes, npts, ids, pos, uv, bad, step10, split.o2);
    if (rc0) return rc0;
    split.fid = fid;
    split.step10 = step10;
    if (begin_only) {
      split.open = true;
      return EAO_OK;
    }
    return frame_tail(out);
  }
  // eao_replay_frame_end: the deferred line association, SampleObjYaw (10.6), the outputs
  int frame_end(int32_t* out) {
    if (!split.open) return EAO_E_STATE;
    split.open = false;
    associate_lines(split.o2, nullptr);
    return frame_tail(out);
  }
  int frame_tail(int32_t* out) {
    Tick tk(&prof[0]);
    const unsigned long fid = split.fid;
    std::vector<Det*>& o2 = split.o2;
    if (split.step10 && yaw_on())  // 10.6 SampleObjYaw for regular objects seen this frame (Tracking.cc:1650-1671)
      for (int i = (int)objs.size() - 1; i >= 0; i--) {
        Obj* o = objs[i].get();
        if (o->bad) continue;
        if ((unsigned long)(long)o->last_add < fid - 5) continue;
        if (!(yaw_class(o->cls) && (unsigned long)(long)o->last_add == fid)) continue;
        if (o->pending) {  // cuboid not final yet: sample when its forest completes
          o->yaw_due = true;
          std::memcpy(o->yawT, pz.T, sizeof(o->yawT));
        } else {
          sample_yaw(o, pz.T);
        }
      }
    for (Det* f : o2) {
      const int k = f->index;
      out[4 * k] = f->method;
      out[4 * k + 1] = f->mnId;
      out[4 * k + 2] = f->cls;
      out[4 * k + 3] = (int)f->pts.size();
    }
    o2.clear();
    if (pend_err) {
      const int e = pend_err;
      pend_err = 0;
      return e;
    }
    return EAO_OK;
  }
  int frame_body(unsigned long fid, const float* Tcw, int nb, const int32_t* boxes, int npts, const int32_t* ids,
                 const float* pos, const float* uv, const uint8_t* bad, bool& step10, std::vector<Det*>& o2) {
    Tick tk(&prof[0]);
    tr(1, (int)fid);
    frame_t0 = now_us();
    phase = 4;
    prof[8] += 1;
    cur = fid;
    std::memcpy(pz.T, Tcw, sizeof(pz.T));
    epoch++;
    kept_cur.clear();
    kept_pos = -1;
    cur_np_done = true;
    np_cache.clear();
    o2.clear();
    std::vector<Det*> kept;
    over.assign(objs.size(), 0);
    if (prep.active && (prep.in.fid != fid || prep.in.nb != nb)) discard_lookahead();  // not the stream's next
    if (prep.active) {  // steps 1-6 (partly) ran ahead, while the previous frame waited on the GPU
      Tick tpf(&prof[56]);
      while (!prep.ok) prep.ok = prep_step(prep);
      o2.swap(prep.o2);
      kept.swap(prep.kept);
      prep.ok = prep.active = false;
      if (prep.took_lines) release_staged_lines();  // its line set is consumed for good
      prep.took_lines = false;
      prep.created.clear();
    } else {
      bool pend = false;  // forests still pending from the previous frame read positions / flags
      for (auto& up : objs) pend |= up->pending != 0;
      for (int i = 0; pend && i < npts; i++) {
        auto it = mp_lookup(ids[i]);
        if (!it) continue;
        const bool nb_ = bad ? bad[i] != 0 : false;
        if (std::memcmp(it->pos, pos + 3 * i, sizeof(float) * 3) != 0 || it->bad != nb_) {
          if (int rc = flush(-1)) return rc;
          pend = false;
        }
      }
      FrameIn in;
      in.fid = fid;
      in.T = Tcw;
      in.nb = nb;
      in.npts = npts;
      in.boxes = boxes;
      in.ids = ids;
      in.pos = pos;
      in.uv = uv;
      in.bad = bad;
      Prep& s = prep_now;
      prep_begin(s, in);
      while (!prep_step(s)) {
      }
      o2.swap(s.o2);
      kept.swap(s.kept);
    }
    double tA = now_us();
    // STEP 9 InitObjMap, Tracking.cc:2531-2598
    if (!ini) {
      int good = -1;
      for (Det* f : kept) {
        if (f->pts.size() < 10) {
          f->method = 6;
          continue;
        }
        good++;
        ini = true;
        ini_frame = (long)fid;
        std::unique_ptr<Obj> o(new Obj());
        o->frames.push_back(f);
        o->id = good;
        o->cls = f->cls;
        o->conf = 1;
        o->last_add = o->lastlast_add = (int)fid;
        o->last = f->box;
        for (int a = 0; a < 3; a++) {
          o->sum[a] = f->sum[a];
          o->center[a] = f->pos[a];
        }
        for (MapPt* p : f->pts) {
          p->vote_insert(o->id, 1);
          o->pts.push_back(p);
        }
        f->mnId = o->id;
        f->method = 7;
        f->alias = o.get();
        mean_std(o.get());
        objs.push_back(std::move(o));
      }
    }
    prof[13] += now_us() - tA;
    tA = now_us();
    // STEP 10
    if ((long)fid > ini_frame && ini) {
      std::vector<Obj*> recent;
      for (auto& up : objs) {
        Obj* o = up.get();
        if (o->bad) continue;
        if ((unsigned long)(long)o->last_add > fid - 30) recent.push_back(o);
        else o->proj = IRect(0, 0, 0, 0);
      }
      // with the NP statistics of every (kept detection, same-class object) pair
      std::vector<std::pair<Det*, Obj*>> pairs;
      std::vector<int> di, oi;
      if (flag != "NA" && flag != "IoU") {
        for (Det* f : kept) {
          if (f->pts.size() < 5) continue;
          for (size_t i = 0; i < objs.size(); i++) {
            Obj* o = objs[i].get();
            if (o->cls != f->cls || o->bad) continue;
            pairs.push_back({f, o});
            di.push_back(f->index);
            oi.push_back((int)i);
          }
        }
      }
      phase = 0;
      int rc = frame_start_gpu(recent, pairs, di, oi);
      phase = 1;
      if (rc) return rc;
      prof[14] += now_us() - tA;
      tA = now_us();
      kept_cur = kept;
      for (size_t q = 0; q < kept.size(); q++) {
        Det* f = kept[q];
        kept_pos = (int)q;
        if (f->pts.size() < 5) {
          f->method = 6;
          continue;
        }
        rc = associate(f);
        if (rc) return rc;
      }
      kept_pos = (int)kept.size();
      cur_np_done = true;
      tr(4);
      prof[15] += now_us() - tA;
      tA = now_us();
      {
        // end of frame: the forests of this frame's updates are launched, not
        // awaited -- each completes at the first read of its object (next
        // frame's step 10 at the latest, or earlier if a point it holds changes)
        Tick tk(&prof[17]);
        rc = kick();
      }
      if (rc) return rc;
      Tick tke(&prof[30]);
      phase = 2;
      for (int i = (int)objs.size() - 1; i >= 0; i--) {  // 10.3
        if (flag == "NA") continue;
        Obj* o = objs[i].get();
        if (o->bad) continue;
        const int df = (int)o->frames.size();
        if (df < 10 && (unsigned long)(long)o->last_add < (fid - 30)) {
          if (df < 5)
            o->bad = true;
          else {
            bool ov = false;
            for (int j = (int)objs.size() - 1; j >= 0; j--) {
              if (objs[j]->bad || i == j) continue;
              // cuboids read: final unless a new object's ComputeMeanAndStandard follows its forest
              if ((o->pending == 2 && (rc = touch(o))) || (objs[j]->pending == 2 && (rc = touch(objs[j].get()))))
                return rc;
              if (overlap(o, objs[j].get())) {
                ov = true;
                break;
              }
            }
            if (ov) o->bad = true;
          }
        }
      }
      for (int i = (int)objs.size() - 1; i >= 0; i--) {  // 10.4
        if ((unsigned long)(long)objs[i]->last_add != fid) continue;
        for (int j = (int)objs.size() - 1; j >= 0; j--) {
          if (i == j) continue;
          if ((unsigned long)(long)objs[j]->last_add == fid) {
            auto& m = objs[i]->same;
            auto it = m.find(objs[j]->id);
            if (it != m.end()) it->second += 1;
            else m[objs[j]->id] = 1;
          }
        }
      }
      step10 = true;  // 10.6 in frame_tail
    }
    return EAO_OK;
  }

  // ---- LocalMapping object maintenance, LocalMapping.cc:772-882
  bool double_ttest(Obj* a, Obj* b) {  // Object.cc:1659-1712 (Q5)
    const int n1 = (int)a->frames.size(), n2 = (int)b->frames.size();
    float t[3];
    for (int k = 0; k < 3; k++) {
      const float m1 = a->center[k], m2 = b->center[k];
      const float d = std::sqrt(((((float)(n1 - 1) * m1 * m1) + ((float)(n2 - 1) * m2 * m2)) /
                                 (float)(n1 + n2 - 2)) * (float)(1 / n1 + 1 / n2));
      t[k] = (m1 - m2) / d;
    }
    const float* row = kTTable[std::min(n1 + n2 - 2, 121)];
    return t[0] < row[5] && t[1] < row[5] && t[2] < row[5];
  }

  void merge(Obj* a, Obj* b) {  // Object_Map::MergeTwoMapObjs, Object.cc:1716-1902
    PosSet& have = posset;
    have.reset(a->pts.size() + b->pts.size());
    for (MapPt* q : a->pts) {
      PosKey k;
      if (pos_key(q->pos, k)) have.insert(k);
    }
    double qi[4], ti[3];
    se3_inverse(a->q, a->t, qi, ti);
    for (MapPt* p : b->pts) {
      const double v[3] = {p->pos[0], p->pos[1], p->pos[2]};
      double s[3];
      se3_apply(qi, ti, v, s);
      if (std::fabs(s[0]) > 1.1 * a->lenth / 2 || std::fabs(s[1]) > 1.1 * a->width / 2 ||
          std::fabs(s[2]) > 1.1 * a->height / 2)
        continue;
      vote(p, a->id);
      PosKey k;
      const bool finite = pos_key(p->pos, k);
      if (!finite || !have.contains(k)) {
        a->pts.push_back(p);
        for (int c = 0; c < 3; c++) a->sum[c] += p->pos[c];
        if (finite) have.insert(k);
      }
    }
    for (Det* f : b->frames) {
      f->mnId = a->id;
      a->conf++;
      a->frames.push_back(f);
    }
    for (auto& kv : b->same) {
      auto it = a->same.find(kv.first);
      if (it != a->same.end()) it->second = it->second + kv.second;
      else a->same[kv.first] = 1;
    }
    const int oLast = a->last_add, oLastLast = a->lastlast_add;
    const IRect oRect = a->last;
    if (a->last_add > b->last_add) {
      if (!(oLastLast > b->last_add)) {
        a->lastlast_add = b->last_add;
        a->lastlast = b->frames.back()->box;
      }
    } else {
      a->last_add = b->last_add;
      a->last = b->frames.back()->box;
      if (oLast > b->lastlast_add) {
        a->lastlast_add = oLast;
        a->lastlast = oRect;
      } else {
        a->lastlast_add = b->lastlast_add;
        a->lastlast = b->frames.size() >= 2 ? b->frames[b->frames.size() - 2]->box : b->frames.front()->box;
      }
    }
    if (yaw_class(a->cls)) {  // step 5. orientation measurements, Object.cc:1842-1901
      for (auto& rr : b->angles) {
        bool fresh = true;
        for (auto& rt : a->angles)
          if (rr[0] == rt[0]) {
            rt[1] += rr[1];
            for (int q = 2; q < 5; q++) rt[q] = rt[q] * ((rt[1] - rr[1]) / rt[1]) + rr[q] * (rr[1] / rt[1]);
            fresh = false;
            break;
          }
        if (fresh) a->angles.push_back(rr);
      }
      if (!a->angles.empty()) {
        int best = 0;
        float best_score = 0.0f;
        for (int i = 0; i < std::min(6, (int)a->angles.size()); i++)
          if (a->angles[i][2] > best_score) {
            best_score = a->angles[i][2];
            best = i;
          }
        a->rotY = a->angles[best][0];
        a->err_par = a->angles[best][3];
        a->err_yaw = a->angles[best][4];
        update_pose(a);
      }
    }
  }

  int iforest_now(Obj* o) {  // synchronous forest (LocalMapping merge path)
    Tick tk(&prof[11]);
    prof[10] += 1;
    o->pending = std::max(o->pending, 1);
    return complete_forest(o);
  }

  int whether_merge(Obj* o) {  // Object_Map::WhetherMergeTwoMapObjs, Object.cc:1607-1655
    for (auto& kv : o->reobj) {
      const int nid = kv.first;
      if (kv.second < 3) continue;
      if (objs[nid]->bad) continue;
      const bool dt = double_ttest(o, objs[nid].get());
      if (o->same.find(nid) != o->same.end()) continue;
      const bool same = false;
      if (!same || dt) {
        Obj* b = objs[nid].get();
        if (o->frames.size() > b->frames.size()) {
          merge(o, b);
          mean_std(o);
          int rc = iforest_now(o);
          if (rc) return rc;
          b->bad = true;
        } else {
          merge(b, o);
          mean_std(b);
          int rc = iforest_now(b);
          if (rc) return rc;
          o->bad = true;
        }
      }
    }
    return EAO_OK;
  }

  void divide_equally(Obj* a, Obj* b, float ox, float oy, float oz) {  // Object.cc:2044-2073
    size_t w = 0;
    for (size_t i = 0; i < a->pts.size(); i++) {
      const float* P = a->pts[i]->pos;
      const bool in =
          (P[0] > b->center_c[0] - (b->lenth / 2 - ox / 2) && P[0] < b->center_c[0] + (b->lenth / 2 - ox / 2)) &&
          (P[1] > b->center_c[1] - (b->width / 2 - oy / 2) && P[1] < b->center_c[1] + (b->width / 2 - oy / 2)) &&
          (P[2] > b->center_c[2] - (b->height / 2 - oz / 2) && P[2] < b->center_c[2] + (b->height / 2 - oz / 2));
      if (!in) a->pts[w++] = a->pts[i];
    }
    a->pts.resize(w);
  }

  void big_to_small(Obj* a, Obj* s) {  // Object.cc:1926-2040
    Tick tbs(&prof[37]);
    double tq = now_us();
    const float box[6] = {s->xmn, s->xmx, s->ymn, s->ymx, s->zmn, s->zmx};
    // the same box over the list it left last time, no point moved since: nothing to erase
    bool given = false;
    if (!(g_ms_memo && a->bts_epoch != ~0ull && std::memcmp(box, a->bts_box, sizeof box) == 0 &&
          a->pts == a->bts_pts && points_unchanged(a, a->bts_epoch))) {
      prof[31] += 1;
      const size_t n = a->pts.size();
      size_t w = 0;
      // the list as ComputeMeanAndStandard last saw it, no point changed since: its positions are
      // cached contiguously, and none of its points is bad
      if (g_ms_memo && a->ms_epoch != ~0ull && n == a->ms_pts.size() && a->ms_pos.size() == 3 * n &&
          (n == 0 || std::memcmp(a->pts.data(), a->ms_pts.data(), sizeof(MapPt*) * n) == 0) &&
          points_unchanged(a, a->ms_epoch)) {
        if (bts_p.size() < 3 * n) bts_p.resize(3 * n + 192);
        const float *X = a->ms_pos.data(), *Y = X + n, *Z = Y + n;
        float* fx = bts_p.data();
        for (size_t i = 0; i < n; i++) {
          const bool in = X[i] > box[0] && X[i] < box[1] && Y[i] > box[2] && Y[i] < box[3] && Z[i] > box[4] &&
                          Z[i] < box[5];
          if (!in) {
            a->pts[w] = a->pts[i];
            fx[w] = X[i];
            fx[n + w] = Y[i];
            fx[2 * n + w] = Z[i];
            w++;
          }
        }
        // blocks of the filtered length for mean_std
        std::memmove(fx + w, fx + n, sizeof(float) * w);
        std::memmove(fx + 2 * w, fx + 2 * n, sizeof(float) * w);
        given = true;
      } else {
        for (size_t i = 0; i < n; i++) {
          const float* P = a->pts[i]->pos;
          const bool in = P[0] > box[0] && P[0] < box[1] && P[1] > box[2] && P[1] < box[3] && P[2] > box[4] &&
                          P[2] < box[5];
          if (!in) a->pts[w++] = a->pts[i];
        }
      }
      a->pts.resize(w);
    }
    prof[38] += now_us() - tq;
    if (given) ms_in = bts_p.data();
    mean_std(a);  // drops bad points only: the list stays clear of the box
    ms_in = nullptr;
    a->bts_epoch = pt_epoch;
    std::memcpy(a->bts_box, box, sizeof box);
    a->bts_pts = a->pts;
  }

  void deal_overlap(Obj* a, Obj* b, float ox, float oy, float oz) {  // Object.cc:2077-2178
    const float va = (a->lenth * a->width) * a->height, vb = (b->lenth * b->width) * b->height;
    const float ov = (ox * oy) * oz;
    const bool bIou = (ov / (va + vb - ov)) >= 0.3;
    const bool bVol = (va > 2 * vb) || (vb > 2 * va);
    bool bSame = false;
    auto it = a->same.find(b->id);
    if (it != a->same.end()) bSame = it->second > 3;
    const bool bCls = a->cls == b->cls;
    if (bIou && !bVol && !bSame && bCls) {
      if (a->frames.size() >= b->frames.size()) {
        merge(a, b);
        b->bad = true;
      } else {
        merge(b, a);
        a->bad = true;
      }
    } else if (bVol && !bSame && bCls) {
      if (a->frames.size() >= b->frames.size() && va > vb) b->bad = true;
      else if (a->frames.size() < b->frames.size() && va < vb) a->bad = true;
    } else if (bIou && !bVol && bSame && bCls) {
      divide_equally(a, b, ox, oy, oz);
      divide_equally(b, b, ox, oy, oz);
      mean_std(a);
      mean_std(b);
    } else if (!bIou && bVol && bSame && !bCls) {
      if (va > vb) big_to_small(a, b);
      else if (va < vb) big_to_small(b, a);
    } else if (bIou && !bSame && bCls) {
      if (a->frames.size() / 2 >= b->frames.size()) {
        merge(a, b);
        b->bad = true;
      } else if (b->frames.size() / 2 >= a->frames.size()) {
        merge(b, a);
        a->bad = true;
      }
    }
  }

  int local_mapping() {
    if (split.open) return EAO_E_STATE;  // the open frame's tail first
    Tick tk(&prof[1]);
    tr(8);
    struct TrEnd {
      ReplayEngine* r;
      ~TrEnd() { r->tr(9); }
    } tr_end{this};
    phase = 3;
    int rc;
    // ComputeMeanAndStandard of every object with >= 10 points (LocalMapping.cc:772-790), after
    // the pending forests complete. An object without a forest in flight is not touched by the
    // flush (a completion changes only its own object's points and cuboid, and other objects'
    // projected rects / reobj votes), so its statistics are computed first, while the forests
    // still run on the GPU; the others after their completion. Same values, same per-object order.
    std::vector<char> ms_done(objs.size(), 0);
    {
      Tick t1(&prof[25]);
      for (size_t i = 0; i < objs.size(); i++) {
        Obj* o = objs[i].get();
        if (o->pending || o->pts.size() < 10 || o->bad) continue;
        mean_std(o);
        ms_done[i] = 1;
      }
    }
    {
      Tick t0(&prof[24]);
      rc = flush(-1);
    }
    if (rc) return rc;
    {
      Tick t1(&prof[25]);
      for (size_t i = 0; i < objs.size(); i++) {
        Obj* o = objs[i].get();
        if (ms_done[i] || o->pts.size() < 10 || o->bad) continue;
        mean_std(o);
      }
    }
    if (flag == "NA" || flag == "IoU" || flag == "NP") return EAO_OK;
    Tick t2(&prof[26]);
    for (auto& up : objs) {
      Obj* o = up.get();
      if (o->bad) continue;
      if (o->frames.size() >= 10 && !o->reobj.empty()) {
        rc = whether_merge(o);
        if (rc) return rc;
      }
    }
    Tick tdo(&prof[29]);
    for (size_t i = 0; i < objs.size(); i++) {
      Obj* a = objs[i].get();
      if (a->pts.size() < 10 || a->bad || a->frames.size() < 10) continue;
      for (size_t j = 0; j < objs.size(); j++) {
        if (i == j) continue;
        Obj* b = objs[j].get();
        if (b->pts.size() < 10 || b->bad || b->frames.size() < 10) continue;
        const float dx = (float)std::fabs(a->center_c[0] - b->center_c[0]);
        const float dy = (float)std::fabs(a->center_c[1] - b->center_c[1]);
        const float dz = (float)std::fabs(a->center_c[2] - b->center_c[2]);
        const float sl = a->lenth / 2 + b->lenth / 2, sw = a->width / 2 + b->width / 2,
                    sh = a->height / 2 + b->height / 2;
        if (dx < sl && dy < sw && dz < sh) deal_overlap(a, b, sl - dx, sw - dy, sh - dz);
      }
    }
    return EAO_OK;
  }
};

}  // namespace eao

using namespace eao;

// One handle is reached from the Tracking thread (eao_replay_frame) and the LocalMapping
// thread (eao_replay_update_points / eao_replay_local_mapping, LocalMapping.cc:86-92):
// every entry point holds the handle's lock, so the calls are serialised in the order the
// threads take it (the reference races there; the engine's containers must not).
// Recursive: eao_replay_run re-enters eao_replay_frame / eao_replay_local_mapping.
struct eao_replay {
  ReplayEngine r;
  std::recursive_mutex mu;
};
#define EAO_REPLAY_LOCK(r) std::lock_guard<std::recursive_mutex> eao_replay_lk_((r)->mu)

extern "C" {

int eao_replay_create(eao_assoc* a, const char* flag, int img_w, int img_h, const float* K4,
                      eao_replay** out) {
  if (!a || !flag || !K4 || !out || img_w <= 0 || img_h <= 0) return EAO_E_ARG;
  std::unique_ptr<eao_replay> r(new eao_replay());
  r->r.A = assoc_engine(a);
  r->r.flag = flag;
  r->r.pz.fx = K4[0];
  r->r.pz.fy = K4[1];
  r->r.pz.cx = K4[2];
  r->r.pz.cy = K4[3];
  r->r.pz.cols = img_w;
  r->r.pz.rows = img_h;
  eao_camera c{img_w, img_h, K4[0], K4[1], K4[2], K4[3]};
  r->r.camdev = make_cam(c);
  r->r.adopt();
  *out = r.release();
  return EAO_OK;
}

// The caller joins every other thread that uses the handle first (eao_accel.h): a lock
// taken here could not keep a late caller out of a freed handle.
int eao_replay_destroy(eao_replay* r) {
  delete r;
  return EAO_OK;
}

int eao_replay_frame(eao_replay* r, int frame_id, const float* Tcw, int n_boxes, const int32_t* boxes,
                     int n_pts, const int32_t* mp_ids, const float* mp_pos, const float* kp_uv,
                     const uint8_t* mp_bad, int32_t* det_out) {
  if (!r || !Tcw || n_boxes < 0 || n_pts < 0 || (n_boxes && (!boxes || !det_out)) ||
      (n_pts && (!mp_ids || !mp_pos || !kp_uv)))
    return EAO_E_ARG;
  EAO_REPLAY_LOCK(r);
  EAO_HIP_CHECK(hipSetDevice(r->r.A->dev));
  const int rc = r->r.frame((unsigned long)frame_id, Tcw, n_boxes, boxes, n_pts, mp_ids, mp_pos, kp_uv,
                            mp_bad, det_out);
  return rc ? rc : (int)r->r.objs.size();
}

int eao_replay_frame_begin(eao_replay* r, int frame_id, const float* Tcw, int n_boxes, const int32_t* boxes,
                           int n_pts, const int32_t* mp_ids, const float* mp_pos, const float* kp_uv,
                           const uint8_t* mp_bad) {
  if (!r || !Tcw || n_boxes < 0 || n_pts < 0 || (n_boxes && !boxes) || (n_pts && (!mp_ids || !mp_pos || !kp_uv)))
    return EAO_E_ARG;
  EAO_REPLAY_LOCK(r);
  EAO_HIP_CHECK(hipSetDevice(r->r.A->dev));
  return r->r.frame((unsigned long)frame_id, Tcw, n_boxes, boxes, n_pts, mp_ids, mp_pos, kp_uv, mp_bad, nullptr,
                    true);
}

int eao_replay_frame_end(eao_replay* r, int32_t* det_out) {
  if (!r) return EAO_E_ARG;
  EAO_REPLAY_LOCK(r);
  if (!r->r.split.open) return EAO_E_STATE;
  if (!r->r.split.o2.empty() && !det_out) return EAO_E_ARG;
  EAO_HIP_CHECK(hipSetDevice(r->r.A->dev));
  const int rc = r->r.frame_end(det_out);
  return rc ? rc : (int)r->r.objs.size();
}

int eao_replay_run(eao_replay* r, int n_frames, const int32_t* frame_ids, const float* Tcw,
                   const int32_t* n_boxes, const int32_t* boxes, const int32_t* n_pts,
                   const int32_t* mp_ids, const float* mp_pos, const float* kp_uv,
                   const uint8_t* mp_bad, const uint8_t* keyframe, int32_t* det_out) {
  return eao_replay_run_updates(r, n_frames, frame_ids, Tcw, n_boxes, boxes, n_pts, mp_ids, mp_pos, kp_uv, mp_bad,
                                keyframe, nullptr, nullptr, nullptr, nullptr, det_out);
}

static int replay_stream(eao_replay* r, int n_frames, const int32_t* frame_ids, const float* Tcw,
                         const int32_t* n_boxes, const int32_t* boxes, const int32_t* n_pts,
                         const int32_t* mp_ids, const float* mp_pos, const float* kp_uv,
                         const uint8_t* mp_bad, const uint8_t* keyframe, const int32_t* n_upd,
                         const int32_t* upd_ids, const float* upd_pos, const uint8_t* upd_bad,
                         int32_t* det_out);

int eao_replay_run_updates(eao_replay* r, int n_frames, const int32_t* frame_ids, const float* Tcw,
                           const int32_t* n_boxes, const int32_t* boxes, const int32_t* n_pts,
                           const int32_t* mp_ids, const float* mp_pos, const float* kp_uv,
                           const uint8_t* mp_bad, const uint8_t* keyframe, const int32_t* n_upd,
                           const int32_t* upd_ids, const float* upd_pos, const uint8_t* upd_bad,
                           int32_t* det_out) {
  if (!r || n_frames < 0 || (n_frames && (!frame_ids || !Tcw || !n_boxes || !n_pts || !keyframe)))
    return EAO_E_ARG;
  if (n_upd) {
    for (int t = 0; t < n_frames; t++)
      if (n_upd[t] < 0) return EAO_E_ARG;
    for (int t = 0; t < n_frames; t++)
      if (n_upd[t] && !upd_ids) return EAO_E_ARG;
  }
  EAO_REPLAY_LOCK(r);
  ReplayEngine& E = r->r;
  E.discard_lookahead();
  const int rc = replay_stream(r, n_frames, frame_ids, Tcw, n_boxes, boxes, n_pts, mp_ids, mp_pos, kp_uv, mp_bad,
                               keyframe, n_upd, upd_ids, upd_pos, upd_bad, det_out);
  if (rc < 0) E.discard_lookahead();  // an aborted stream leaves no look-ahead behind
  return rc;
}

static int replay_stream(eao_replay* r, int n_frames, const int32_t* frame_ids, const float* Tcw,
                         const int32_t* n_boxes, const int32_t* boxes, const int32_t* n_pts,
                         const int32_t* mp_ids, const float* mp_pos, const float* kp_uv,
                         const uint8_t* mp_bad, const uint8_t* keyframe, const int32_t* n_upd,
                         const int32_t* upd_ids, const float* upd_pos, const uint8_t* upd_bad,
                         int32_t* det_out) {
  size_t ob = 0, op = 0, ou = 0;
  ReplayEngine& E = r->r;
  for (int t = 0; t < n_frames; t++) {
    // the next frame's inputs, for the look-ahead of steps 1-6 (not across a point record)
    E.la_set = false;
    // (only for well-formed counts: a malformed next frame is refused by its own call)
    if (t + 1 < n_frames && !(n_upd && n_upd[t]) && n_boxes[t + 1] >= 0 && n_pts[t + 1] >= 0) {
      ReplayEngine::FrameIn& in = E.la;
      in.fid = (unsigned long)frame_ids[t + 1];
      in.T = Tcw + 16 * (size_t)(t + 1);
      in.nb = n_boxes[t + 1];
      in.npts = n_pts[t + 1];
      in.boxes = boxes + 5 * (ob + (size_t)n_boxes[t]);
      const size_t op1 = op + (size_t)n_pts[t];
      in.ids = mp_ids + op1;
      in.pos = mp_pos + 3 * op1;
      in.uv = kp_uv + 2 * op1;
      in.bad = mp_bad ? mp_bad + op1 : nullptr;
      E.la_set = true;
    }
    const int rc = eao_replay_frame(r, frame_ids[t], Tcw + 16 * (size_t)t, n_boxes[t], boxes + 5 * ob, n_pts[t],
                                    mp_ids + op, mp_pos + 3 * op, kp_uv + 2 * op, mp_bad ? mp_bad + op : nullptr,
                                    det_out + 4 * ob);
    if (rc < 0) return rc;
    if (n_upd && n_upd[t]) {  // the frame's map-point record (LocalBA / culling / fuse)
      const int ru = eao_replay_update_points(r, n_upd[t], upd_ids + ou, upd_pos ? upd_pos + 3 * ou : nullptr,
                                              upd_bad ? upd_bad + ou : nullptr);
      if (ru < 0) return ru;
      ou += (size_t)n_upd[t];
    }
    if (keyframe[t]) {
      const int rl = eao_replay_local_mapping(r);
      if (rl < 0) return rl;
    }
    ob += (size_t)n_boxes[t];
    op += (size_t)n_pts[t];
  }
  E.la_set = false;
  if (E.prep.active) {
    eao::set_error("replay: look-ahead frame left unconsumed");
    return EAO_E_STATE;
  }
  // the stream's last forests complete here, inside the call (no work left pending for a
  // later reader)
  EAO_HIP_CHECK(hipSetDevice(r->r.A->dev));
  if (int rc = r->r.flush(-1)) return rc;
  return (int)r->r.objs.size();
}

int eao_replay_update_points(eao_replay* r, int n, const int32_t* ids, const float* pos, const uint8_t* bad) {
  if (!r || n < 0 || (n && !ids)) return EAO_E_ARG;
  EAO_REPLAY_LOCK(r);
  EAO_HIP_CHECK(hipSetDevice(r->r.A->dev));
  return r->r.update_points(n, ids, pos, bad);
}

int eao_replay_held_points(eao_replay* r, int32_t* ids, int cap) {
  if (!r || cap < 0 || (cap && !ids)) return EAO_E_ARG;
  EAO_REPLAY_LOCK(r);
  std::vector<int32_t> v;
  const int n = r->r.held_points(v);
  if (n > 0 && cap > 0) std::memcpy(ids, v.data(), sizeof(int32_t) * (size_t)std::min(n, cap));
  return n;
}

int eao_replay_lines(eao_replay* r, int n_frames, const int32_t* n_lines, const float* lines) {
  if (!r || n_frames < 0 || (n_frames && (!n_lines || !lines))) return EAO_E_ARG;
  EAO_REPLAY_LOCK(r);
  for (int t = 0; t < n_frames; t++) {
    if (n_lines[t] < 0) return EAO_E_ARG;
    r->r.staged_lines.emplace_back(lines, lines + 4 * (size_t)n_lines[t]);
    lines += 4 * (size_t)n_lines[t];
  }
  return EAO_OK;
}

int eao_replay_local_mapping(eao_replay* r) {
  if (!r) return EAO_E_ARG;
  EAO_REPLAY_LOCK(r);
  EAO_HIP_CHECK(hipSetDevice(r->r.A->dev));
  return r->r.local_mapping();
}

int eao_replay_profile(eao_replay* r, double* out24) {
  if (!r || !out24) return EAO_E_ARG;
  EAO_REPLAY_LOCK(r);
  std::memcpy(out24, r->r.prof, sizeof(double) * 24);
  return EAO_OK;
}

int eao_replay_profile_n(eao_replay* r, double* out, int n) {
  if (!r || !out || n < 0) return EAO_E_ARG;
  EAO_REPLAY_LOCK(r);
  std::memcpy(out, r->r.prof, sizeof(double) * std::min(n, 60));
  return std::min(n, 60);
}

}  // extern "C"

namespace {
struct CallbackExchanger : eao::Exchanger {
  eao_allgather_fn fn;
  void* ctx;
  CallbackExchanger(eao_allgather_fn f, void* c) : fn(f), ctx(c) {}
  int allgather(const void* send, void* recv, size_t bytes) override {
    const int rc = fn(ctx, send, recv, bytes);
    if (rc) eao::set_error("replay: all-gather callback failed");
    return rc ? EAO_E_ARG : EAO_OK;
  }
};
int shard_check(eao_replay* r, int rank, int world) {
  if (!r || world < 1 || rank < 0 || rank >= world) return EAO_E_ARG;
  if (!r->r.objs.empty() || r->r.ini) {
    eao::set_error("replay: sharding must be set before the first frame");
    return EAO_E_ARG;
  }
  return EAO_OK;
}
}  // namespace

extern "C" {

int eao_replay_shard_callback(eao_replay* r, int rank, int world, eao_allgather_fn fn, void* ctx) {
  if (!r) return EAO_E_ARG;
  EAO_REPLAY_LOCK(r);
  if (int rc = shard_check(r, rank, world)) return rc;
  if (world > 1 && !fn) return EAO_E_ARG;
  r->r.ex.reset(world > 1 ? new CallbackExchanger(fn, ctx) : nullptr);
  r->r.srank = rank;
  r->r.sworld = world;
  return EAO_OK;
}

int eao_replay_shard_rccl(eao_replay* r, int rank, int world, const uint8_t* unique_id) {
  if (!r) return EAO_E_ARG;
  EAO_REPLAY_LOCK(r);
  if (int rc = shard_check(r, rank, world)) return rc;
  if (!unique_id) return EAO_E_ARG;
  int rc = EAO_OK;
  eao::Exchanger* x = eao::make_rccl_exchanger(r->r.A->dev, rank, world, unique_id, &rc);
  if (!x) return rc ? rc : EAO_E_HIP;
  r->r.ex.reset(x);
  r->r.srank = rank;
  r->r.sworld = world;
  return EAO_OK;
}

int eao_replay_shard_stats(eao_replay* r, double* out3) {
  if (!r || !out3) return EAO_E_ARG;
  EAO_REPLAY_LOCK(r);
  std::memcpy(out3, r->r.xstat, sizeof(double) * 3);
  return EAO_OK;
}

int eao_replay_num_objects(eao_replay* r) {
  if (!r) return EAO_E_ARG;
  EAO_REPLAY_LOCK(r);
  return (int)r->r.objs.size();
}

int eao_replay_object(eao_replay* r, int i, int32_t* ints, float* floats) {
  if (!r || !ints || !floats) return EAO_E_ARG;
  EAO_REPLAY_LOCK(r);
  if (i < 0 || i >= (int)r->r.objs.size()) return EAO_E_ARG;
  EAO_HIP_CHECK(hipSetDevice(r->r.A->dev));
  int rc = r->r.flush(-1);
  if (rc) return rc;
  const Obj* o = r->r.objs[i].get();
  ints[0] = o->id;
  ints[1] = o->cls;
  ints[2] = o->bad;
  ints[3] = (int)o->frames.size();
  ints[4] = (int)o->pts.size();
  ints[5] = o->last_add;
  ints[6] = (int)o->reobj.size();
  ints[7] = (int)o->same.size();
  for (int a = 0; a < 3; a++) {
    floats[a] = o->center[a];
    floats[3 + a] = o->sd[a];
    floats[6 + a] = o->csd[a];
  }
  floats[9] = o->lenth;
  floats[10] = o->width;
  floats[11] = o->height;
  floats[12] = o->rmax;
  floats[13] = o->csd_all;
  floats[14] = (float)o->proj.x;
  floats[15] = (float)o->proj.w;
  floats[16] = o->rotY;
  floats[17] = (float)o->angles.size();
  floats[18] = o->err_par;
  floats[19] = o->err_yaw;
  return EAO_OK;
}

int eao_replay_object_points(eao_replay* r, int i, int32_t* ids, int cap) {
  if (!r) return EAO_E_ARG;
  EAO_REPLAY_LOCK(r);
  if (i < 0 || i >= (int)r->r.objs.size()) return EAO_E_ARG;
  EAO_HIP_CHECK(hipSetDevice(r->r.A->dev));
  int rc = r->r.flush(-1);
  if (rc) return rc;
  const Obj* o = r->r.objs[i].get();
  const int n = (int)o->pts.size();
  for (int k = 0; k < n && k < cap; k++) ids[k] = o->pts[k]->id;
  return n;
}

}  // extern "C"
