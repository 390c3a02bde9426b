// orb.h -- ORB extraction engine (host side of orb.hip).
#pragma once
#include "common.h"
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../../include/eao_accel.h"

namespace eao {

// same layout as eao_keypoint / cv::KeyPoint
struct eao_keypoint_dev {
  float x, y, size, angle, response;
  int32_t octave, class_id;
};
static_assert(sizeof(eao_keypoint_dev) == sizeof(eao_keypoint), "keypoint layout");

// Per pyramid level geometry (ORBextractor.cc:765-853, :1107-1132)
struct LevelDev {
  int w, h, pitch;
  int pad0;
  long long plane_off;        // byte offset of the level plane in a frame's pyramid area
  int minBX, minBY, maxBX, maxBY;
  int nCols, nRows, wCell, hCell;
  int nfeat;                  // mnFeaturesPerLevel
  int cell_begin, cell_count;
  int cand_off, cand_cap;     // candidate slots (uint32) of this level in a frame
  int sel_off, sel_cap;       // selected keypoint slots of this level in a frame
  int nIni;                   // initial quadtree nodes
  float hX;
  float scale, size;          // mvScaleFactor[l], PATCH_SIZE*scale truncated
  int tab_x, tab_y, xmax;     // resize tables
  int pad1;
};

struct BandDev {              // one row of FAST cells of a level
  int16_t level, ncells;
  int16_t x0, y0, x1, y1;     // union of the cells' ROIs
  int cell_begin;
};

struct CellDev {
  int16_t level, i, j, pad;
  int16_t x0, y0, x1, y1;     // ROI in level coordinates
  int slot;                   // first candidate slot in the frame's candidate area
  int cap;                    // NMS bound on corners in this cell
};

class OrbEngine {
 public:
  eao_orb_params p{};
  int dev = 0;
  std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
  std::vector<int> quotas, umax, gk;
  std::vector<LevelDev> levels;
  std::vector<CellDev> cells;
  std::vector<int> resize_xofs, resize_yrows;
  std::vector<short> resize_ia, resize_ib;
  struct ResizePlan {          // k_resize_lds launch of a level >= 1
    int tr, block, tiles;
    size_t lds;
  };
  std::vector<ResizePlan> resize_plan;
  // levels [tail_a, nlevels) made by one k_pyr_tail launch (tail_a = nlevels: none); its LDS images
  // at 0 and tail_img_b, tail_lds bytes in all
  int tail_a = 0, tail_img_b = 0, tail_tab_b = 0, tail_nx = 0, tail_ny = 0;
  int tail_min_frames = 128;  // smaller batches keep per-level launches (eao_orb_debug_pyramid: 1)
  size_t tail_lds = 0;
  std::vector<int2> slot_map;
  long long pyr_bytes = 0, cand_stride = 0, sel_stride = 0;
  std::vector<BandDev> bands;
  int band_w = 0, band_h = 0;  // largest band ROI
  int cap = 0, roi_stride = 0, roi_rows = 0;
  // optional per-stage timing: events around resize / fast / distribute / describe (blur fused)
  static constexpr int kStages = 4;
  bool timing = false;
  hipEvent_t ev[kStages + 1] = {};

  hipStream_t stream = nullptr;
  LevelDev* d_levels = nullptr;
  CellDev* d_cells = nullptr;
  int *d_xofs = nullptr, *d_yrows = nullptr, *d_umax = nullptr, *d_gk = nullptr;
  short *d_ia = nullptr, *d_ib = nullptr;
  int2* d_slot_map = nullptr;
  uint8_t* d_pyr = nullptr;
  BandDev* d_bands = nullptr;
  uint32_t *d_cand = nullptr, *d_qbuf = nullptr, *d_sel = nullptr;
  int *d_cell_cnt = nullptr, *d_sel_cnt = nullptr;
  uint8_t* d_img = nullptr;
  eao_keypoint_dev* d_out_kps = nullptr;
  uint8_t* d_out_desc = nullptr;
  int* d_out_cnt = nullptr;
  uint8_t* d_out_blk = nullptr;  // the three single-image outputs above, one allocation
  size_t out_kps_off = 0, out_desc_off = 0, out_bytes = 0;
  HostStage stage_in, stage_out;  // single-image staging (pinned image in, outputs back)

  int plan(const eao_orb_params& prm, int device);
  int init(const eao_orb_params& prm, int device);
  int run(const uint8_t* d_frames, int nframes, int pitch, eao_keypoint_dev* d_kps, uint8_t* d_desc,
          int* d_counts, int out_cap, hipStream_t s);
  // single-image calls: the staged image into d_img and the outputs (count, then count keypoints and
  // descriptors) into stage_out by kernel on `stream` (no copy-engine transfers)
  int image_in(size_t bytes);
  int outputs_out();
  ~OrbEngine();
};

// cvtColor(CV_{RGB,BGR}[A]2GRAY) of a batch of HBM-resident frames (orb.hip)
int color_to_gray(const uint8_t* d_src, int nframes, int w, int h, int spitch, int cn, int rgb, uint8_t* d_dst,
                  int dpitch, hipStream_t s);

}  // namespace eao
