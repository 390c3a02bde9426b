// match.h -- ORB matching engine (host side of match.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/eao_accel.h"
#include "common.h"
#include "orb.h"

namespace eao {

constexpr int GRID_COLS = 64;  // FRAME_GRID_COLS, include/Frame.h:55
constexpr int GRID_ROWS = 48;  // FRAME_GRID_ROWS, include/Frame.h:54
constexpr int GRID_CELLS = GRID_COLS * GRID_ROWS;

struct CamDev {
  float fx, fy, cx, cy;
  float minX, maxX, minY, maxY;  // Frame::mnMinX.. (k1 == 0: 0..w, 0..h)
  float invW, invH;              // mfGridElementWidthInv / HeightInv
};

CamDev make_cam(const eao_camera& c);

class MatchEngine {
 public:
  int dev = 0, max_kps = 0, max_batch = 0;
  hipStream_t stream = nullptr;
  // per-frame-slot grid (CSR), batch sized
  int* d_gstart = nullptr;  // [batch][GRID_CELLS+1]
  int* d_gitems = nullptr;  // [batch][max_kps]
  // single-call staging (2 frames)
  eao_keypoint_dev* d_kps = nullptr;  // [2][max_kps]
  uint8_t* d_desc = nullptr;          // [2][max_kps*32]
  uint8_t* d_u8 = nullptr;            // [max_kps] flags
  float* d_f = nullptr;               // [max_kps*3] positions / misc floats
  float* d_f2 = nullptr;              // [max_kps*3]
  float* d_f3 = nullptr;
  float* d_f4 = nullptr;
  uint8_t* d_mdesc = nullptr;         // [max_kps*32] map point descriptors
  int* d_i32 = nullptr;               // [max_kps] misc ints
  int* d_i32b = nullptr;              // [max_kps]
  int* d_out = nullptr;               // [max_kps + 16]
  float* d_T = nullptr;               // [16 * batch]
  float* d_scales = nullptr;          // [32]
  float* d_geo = nullptr;             // [max_kps][4] per-map-point projection (keyframe search)
  // motion search candidates: MK smallest keys / rotation bins / count per (pair, query)
  unsigned long long* d_ckeys = nullptr;
  signed char* d_cbins = nullptr;
  int* d_ccnt = nullptr;
  HostStage stage, res;  // single-call inputs (pinned image + device mirror) / results (pinned)

  int init(int device, int max_kps, int max_batch);
  ~MatchEngine();
  int build_grid(const CamDev& cam, const eao_keypoint_dev* kps, const int* counts, int n_single,
                 int cap, int nframes, hipStream_t s);
  int motion(const CamDev& cd, const float* d_T, float th, int check_ori, const eao_keypoint_dev* d_kps,
             const uint8_t* d_desc, const int* d_counts, int cap, const uint8_t* d_has, const float* d_pos,
             const uint8_t* d_mdesc, const float* d_sc, int nframes, int* d_match, int* d_nm, hipStream_t s);
};

}  // namespace eao
