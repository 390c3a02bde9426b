// assoc.h -- EAO association engine (host side of assoc.hip / replay.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../../include/eao_accel.h"
#include "hsa_lane.h"
#include "match.h"

namespace eao {

constexpr int NP_MAXN = 8192;   // object points per NP pair handled in LDS
constexpr int IF_MAXN = 7168;   // points per isolation-forest cloud (tree + sample in LDS)
constexpr int IF_CTL = 256;     // CalculateC(leaf size) table entries staged in the forest kernel's LDS
constexpr int IF_TAB_N = 4096;  // cloud sizes covered by the forest's sample table (k_iforest_sample)
constexpr int IF_JSLOTS = 16;   // forest kernel: rank subtrees prepared ahead by helper waves (slots)
constexpr int IF_HELPERS = 3;   // ... and the helper waves (1..3: the other SIMDs of wave 0's CU)
constexpr int IF_TAB_TW = 5;    // generator states per tree in the table: after 1 .. IF_TAB_TW twists
constexpr int IF_LDS = 160 * 1024;  // LDS per workgroup on gfx950

class AssocEngine {
 public:
  int dev = 0, max_points = 0;
  hipStream_t stream = nullptr;
  // staging
  float* d_pts = nullptr;        // [2 * max_points * 3]
  uint8_t* d_valid = nullptr;    // [2 * max_points]
  int* d_meta = nullptr;         // [8 * max_pairs]
  eao_np_stats* d_np = nullptr;  // [max_pairs]
  int* d_rect = nullptr;         // [4 * max_pairs]
  uint8_t* d_ok = nullptr;
  float* d_T = nullptr;
  // isolation forest scratch
  uint32_t* d_mtinit = nullptr;  // [trees][624] mt19937 state of each tree after the first twist
  double* d_contrib = nullptr;   // [max_trees][max_points] path length per (tree, point)
  double* d_ctab = nullptr;      // [IF_MAXN + 1] CalculateC(n) table (leaf sizes, sample sizes)
  uint32_t cached_seed = 0, cached_trees = 0;
  // the sample table (k_iforest_sample): for n in [2, tab_n], sample n / 2, of (cached_seed,
  // cached_trees); built with the generator states, tab_n = 0 until then
  int tab_n = 0;
  uint16_t* d_tab_ids = nullptr;      // per n, per tree: n / 2 sample ids
  long long* d_tab_off = nullptr;     // [IF_TAB_N + 1] offset of size n's block in d_tab_ids
  int* d_tab_D = nullptr;             // [IF_TAB_N + 1][trees] draws taken by the shuffle (-1: not covered)
  uint32_t* d_tab_states = nullptr;   // [trees][IF_TAB_TW][624] states after 1 .. IF_TAB_TW twists
  int iforest_table(uint32_t seed, uint32_t trees, hipStream_t s);
  size_t lds_limit = 0;
  double* d_scores = nullptr;    // [max_points]
  // the erase decision of IsolationForestDeleteOutliers, score > th (th = 0.6f, or 0.65f
  // for class 62), taken exactly as glibc's pow would: x = -E[h]/c(psi) >= pow_x0[k]
  double pow_x0[2] = {0, 0};
  int max_pairs = 256, max_clouds = 64, max_trees = 64;
  // resources a finished association replay hands to the next one on this
  // engine (forest batch slots, streams, pinned staging; opaque, replay.cpp)
  void* replay_pool = nullptr;
  void (*replay_pool_free)(void*) = nullptr;

  int init(int device, int max_points);
  ~AssocEngine();
  // device-level entry points (inputs already on device, launched on lane s: a HIP stream or an
  // HSA queue, hsa_lane.h)
  int np_batch(int npairs, const float* d_fp, const uint8_t* d_fv, const int* d_foff,
               const int* d_flen, const float* d_op, const uint8_t* d_ov, const int* d_ooff,
               const int* d_olen, eao_np_stats* d_out, const Lane& s, int max_olen,
               // per pair: the device scores of the object's pending forest (null: none) and its
               // erase threshold -- the erasure is applied on the fly
               const double* const* d_os_ptr = nullptr, const float* d_oth = nullptr);
  int iforest_batch(int nclouds, const float* d_pts, const int* d_off, const int* d_len,
                    uint32_t trees, uint32_t seed, const uint32_t* d_sample, double* d_scores,
                    const Lane& s, int max_len, int max_sample, int npts_total,
                    double* contrib = nullptr,   // [trees][npts_total] scratch, default d_contrib
                    double* scores2 = nullptr,   // optional second copy of the scores
                    // sharded, device form: also each cloud's outlier bit mask into pdst, as pack_masks
                    // (pk = the pack meta [3 nclouds], pth = the thresholds)
                    const int* pk = nullptr, const float* pth = nullptr, unsigned char* pdst = nullptr);
  // on HSA lane s, after the launches before it: zero [zero, zero + zero_bytes) (may be empty),
  // then store v into *flag (the sharded exchange's GPU-side ready flag, shard.h ExReady)
  int publish(const Lane& s, void* zero, size_t zero_bytes, uint64_t* flag, uint64_t v);
  // host (pinned) to device copy as a kernel on stream s (16-byte aligned buffers)
  int stage_in(void* d_dst, const void* h_src, size_t bytes, const Lane& s);
  // can one k_iforest_tree workgroup hold a cloud of max_len points, max_sample samples
  bool iforest_fits(int max_len, int max_sample) const;
  // the frame start's projected rects and NP pairs in one launch (k_rects_np); the inputs
  // may be pinned host memory read in place
  int rects_np(const CamDev& cam, const float* T, int nclouds, const float* rpts, const int* roff, const int* rlen,
               int* rect, uint8_t* ok, const double* const* ros, const float* rth, int npairs, const float* fp,
               const uint8_t* fv, const int* foff, const int* flen, const float* op, const uint8_t* ov,
               const int* ooff, const int* olen, eao_np_stats* out, const Lane& s, int max_olen,
               const double* const* os_ptr, const float* oth);
  int rects(const CamDev& cam, const float* d_T, int nclouds, const float* d_pts, const int* d_off,
            const int* d_len, int* d_rect, uint8_t* d_ok, hipStream_t s,
            const double* const* d_os_ptr = nullptr, const float* d_oth = nullptr);
};

AssocEngine* assoc_engine(eao_assoc* a);

}  // namespace eao
