/*
 * match_ref.cpp -- CPU restatement of the Frame grid and ORBmatcher searches
 * (TEST INFRASTRUCTURE ONLY).  Reference files: src/Frame.cc:351-513,
 * src/ORBmatcher.cc:37-137,405-520,1328-1663, src/MapPoint.cc:373-394.
 */
#include "oracle.h"

#include <algorithm>
#include <climits>
#include <cmath>
#include <vector>

namespace orc {

static const int FRAME_GRID_ROWS = 48;  // include/Frame.h:54
static const int FRAME_GRID_COLS = 64;  // include/Frame.h:55
static const int TH_HIGH = 100, TH_LOW = 50, HISTO_LENGTH = 30;  // ORBmatcher.cc:37-39

struct Grid {
  float minX, maxX, minY, maxY, invW, invH;
  std::vector<int> cells[FRAME_GRID_COLS][FRAME_GRID_ROWS];
};

// Frame::ComputeImageBounds (k1 == 0 branch, Frame.cc:584-590) + grid setup :170-171
static void grid_build(const orc_camera* cam, int n, const orc_keypoint* kps, Grid& g) {
  g.minX = 0.0f;
  g.maxX = (float)cam->img_w;
  g.minY = 0.0f;
  g.maxY = (float)cam->img_h;
  g.invW = (float)FRAME_GRID_COLS / (g.maxX - g.minX);
  g.invH = (float)FRAME_GRID_ROWS / (g.maxY - g.minY);
  // AssignFeaturesToGrid + PosInGrid, Frame.cc:351-366, :503-513
  for (int i = 0; i < n; i++) {
    int px = (int)std::round((kps[i].x - g.minX) * g.invW);
    int py = (int)std::round((kps[i].y - g.minY) * g.invH);
    if (px < 0 || px >= FRAME_GRID_COLS || py < 0 || py >= FRAME_GRID_ROWS) continue;
    g.cells[px][py].push_back(i);
  }
}

// Frame::GetFeaturesInArea, Frame.cc:448-501
static void features_in_area(const Grid& g, const orc_keypoint* kps, float x, float y, float r,
                             int minLevel, int maxLevel, std::vector<int>& out) {
  out.clear();
  const int nMinCellX = std::max(0, (int)std::floor((x - g.minX - r) * g.invW));
  if (nMinCellX >= FRAME_GRID_COLS) return;
  const int nMaxCellX = std::min(FRAME_GRID_COLS - 1, (int)std::ceil((x - g.minX + r) * g.invW));
  if (nMaxCellX < 0) return;
  const int nMinCellY = std::max(0, (int)std::floor((y - g.minY - r) * g.invH));
  if (nMinCellY >= FRAME_GRID_ROWS) return;
  const int nMaxCellY = std::min(FRAME_GRID_ROWS - 1, (int)std::ceil((y - g.minY + r) * g.invH));
  if (nMaxCellY < 0) return;
  const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
  for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
    for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
      const std::vector<int>& cell = g.cells[ix][iy];
      for (int idx : cell) {
        const orc_keypoint& kp = kps[idx];
        if (bCheckLevels) {
          if (kp.octave < minLevel) continue;
          if (maxLevel >= 0 && kp.octave > maxLevel) continue;
        }
        const float distx = kp.x - x, disty = kp.y - y;
        if (std::fabs(distx) < r && std::fabs(disty) < r) out.push_back(idx);
      }
    }
}

// ORBmatcher::DescriptorDistance, ORBmatcher.cc:1647-1663 (SWAR popcount)
int descriptor_distance(const uint8_t* a, const uint8_t* b) {
  const uint32_t* pa = (const uint32_t*)a;
  const uint32_t* pb = (const uint32_t*)b;
  int dist = 0;
  for (int i = 0; i < 8; i++) {
    uint32_t v = pa[i] ^ pb[i];
    v = v - ((v >> 1) & 0x55555555);
    v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
    dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
  }
  return dist;
}

// cv::Mat 3x3 * 3x1 + 3x1 (CV_32F): OpenCV 3.2 gemm small-size path
// (len == 3 == d_size.height): float dot, then (float)(t*1.0 + c*1.0) in double.
static inline void transform_point(const float* T, const float* P, float* out) {
  for (int r = 0; r < 3; r++) {
    float t = T[4 * r] * P[0] + T[4 * r + 1] * P[1] + T[4 * r + 2] * P[2];
    out[r] = (float)((double)t + (double)T[4 * r + 3]);
  }
}

// ORBmatcher::ComputeThreeMaxima, ORBmatcher.cc:1601-1642
static void three_maxima(const std::vector<int>* histo, int L, int& ind1, int& ind2, int& ind3) {
  int max1 = 0, max2 = 0, max3 = 0;
  for (int i = 0; i < L; i++) {
    const int s = (int)histo[i].size();
    if (s > max1) {
      max3 = max2; max2 = max1; max1 = s;
      ind3 = ind2; ind2 = ind1; ind1 = i;
    } else if (s > max2) {
      max3 = max2; max2 = s;
      ind3 = ind2; ind2 = i;
    } else if (s > max3) {
      max3 = s;
      ind3 = i;
    }
  }
  if (max2 < 0.1f * (float)max1) {
    ind2 = -1;
    ind3 = -1;
  } else if (max3 < 0.1f * (float)max1) {
    ind3 = -1;
  }
}

static inline int rot_bin(float a_last, float a_cur) {
  const float factor = 1.0f / HISTO_LENGTH;
  float rot = a_last - a_cur;
  if (rot < 0.0) rot += 360.0f;
  int bin = (int)std::round(rot * factor);
  if (bin == HISTO_LENGTH) bin = 0;
  return bin;
}

}  // namespace orc

using namespace orc;

extern "C" {

int orc_descriptor_distance(const uint8_t* a, const uint8_t* b) { return descriptor_distance(a, b); }

// ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono=true), :1328-1470
int orc_search_by_projection_motion(const orc_camera* cam, const float* Tcw, float th, int check_ori,
                                    int n_last, const orc_keypoint* last_kps,
                                    const uint8_t* last_has_mp, const float* last_mp_pos,
                                    const uint8_t* last_mp_desc, int n_cur,
                                    const orc_keypoint* cur_kps, const uint8_t* cur_desc, int nlevels,
                                    const float* scale_factors, int32_t* cur_match) {
  Grid* g = new Grid();
  grid_build(cam, n_cur, cur_kps, *g);
  for (int i = 0; i < n_cur; i++) cur_match[i] = -1;
  int nmatches = 0;
  std::vector<int> rotHist[HISTO_LENGTH];
  std::vector<int> cand;
  for (int i = 0; i < n_last; i++) {
    if (!last_has_mp[i]) continue;
    float x3Dc[3];
    transform_point(Tcw, last_mp_pos + 3 * i, x3Dc);
    const float xc = x3Dc[0], yc = x3Dc[1];
    const float invzc = (float)(1.0 / x3Dc[2]);
    if (invzc < 0) continue;
    float u = cam->fx * xc * invzc + cam->cx;
    float v = cam->fy * yc * invzc + cam->cy;
    if (u < g->minX || u > g->maxX) continue;
    if (v < g->minY || v > g->maxY) continue;
    int nLastOctave = last_kps[i].octave;
    float radius = th * scale_factors[nLastOctave];
    features_in_area(*g, cur_kps, u, v, radius, nLastOctave - 1, nLastOctave + 1, cand);
    if (cand.empty()) continue;
    const uint8_t* dMP = last_mp_desc + 32 * (size_t)i;
    int bestDist = 256, bestIdx2 = -1;
    for (int i2 : cand) {
      if (cur_match[i2] >= 0) continue;  // mvpMapPoints[i2] && Observations()>0
      const int dist = descriptor_distance(dMP, cur_desc + 32 * (size_t)i2);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx2 = i2;
      }
    }
    if (bestDist <= TH_HIGH) {
      cur_match[bestIdx2] = i;
      nmatches++;
      if (check_ori) rotHist[rot_bin(last_kps[i].angle, cur_kps[bestIdx2].angle)].push_back(bestIdx2);
    }
  }
  (void)nlevels;
  if (check_ori) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
    for (int i = 0; i < HISTO_LENGTH; i++) {
      if (i != ind1 && i != ind2 && i != ind3) {
        for (int idx : rotHist[i]) {
          cur_match[idx] = -1;
          nmatches--;
        }
      }
    }
  }
  delete g;
  return nmatches;
}

// Frame::isInFrustum (Frame.cc:390-446) + MapPoint::PredictScale (MapPoint.cc:385-394)
int orc_is_in_frustum(const orc_camera* cam, const float* Tcw, int n_mp, const float* mp_pos,
                      const float* mp_normal, const float* mp_min_dist, const float* mp_max_dist,
                      float view_cos_limit, float log_scale_factor, uint8_t* in_view, float* proj_xy,
                      int32_t* pred_level, float* view_cos) {
  // mOw = -Rcw^T * tcw (Frame::UpdatePoseMatrices, Frame.cc:384). A transposed
  // operand (GEMM_1_T) leaves OpenCV's small-size path, so GEMMSingleMul
  // accumulates in double and scales by alpha=-1 before rounding to float.
  float Ow[3];
  for (int c = 0; c < 3; c++) {
    double s = (double)Tcw[c] * Tcw[3];
    s += (double)Tcw[4 + c] * Tcw[7];
    s += (double)Tcw[8 + c] * Tcw[11];
    Ow[c] = (float)(s * -1.0);
  }
  int cnt = 0;
  for (int i = 0; i < n_mp; i++) {
    in_view[i] = 0;
    const float* P = mp_pos + 3 * i;
    float Pc[3];
    transform_point(Tcw, P, Pc);
    if (Pc[2] < 0.0f) continue;
    const float invz = 1.0f / Pc[2];
    const float u = cam->fx * Pc[0] * invz + cam->cx;
    const float v = cam->fy * Pc[1] * invz + cam->cy;
    if (u < 0.0f || u > (float)cam->img_w) continue;
    if (v < 0.0f || v > (float)cam->img_h) continue;
    const float maxDistance = 1.2f * mp_max_dist[i];
    const float minDistance = 0.8f * mp_min_dist[i];
    float PO[3] = {P[0] - Ow[0], P[1] - Ow[1], P[2] - Ow[2]};
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)PO[k] * PO[k];
    const float dist = (float)std::sqrt(s);
    if (dist < minDistance || dist > maxDistance) continue;
    const float* Pn = mp_normal + 3 * i;
    double dot = 0;
    for (int k = 0; k < 3; k++) dot += (double)PO[k] * Pn[k];
    const float viewCos = (float)(dot / dist);
    if (viewCos < view_cos_limit) continue;
    float ratio = mp_max_dist[i] / dist;
    // log(float) resolves to logf; defined as the correctly rounded value (Q26)
    int level = (int)std::ceil((float)std::log((double)ratio) / log_scale_factor);
    in_view[i] = 1;
    proj_xy[2 * i] = u;
    proj_xy[2 * i + 1] = v;
    pred_level[i] = level;
    view_cos[i] = viewCos;
    cnt++;
  }
  return cnt;
}

// ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th), :45-129
int orc_search_by_projection_local(const orc_camera* cam, float th, float nnratio, int n_mp,
                                   const uint8_t* in_view, const float* proj_xy,
                                   const int32_t* pred_level,
                                   const float* view_cos, const uint8_t* mp_desc, int n_cur,
                                   const orc_keypoint* cur_kps, const uint8_t* cur_desc,
                                   const int32_t* cur_preassigned, int nlevels,
                                   const float* scale_factors, int32_t* cur_match) {
  Grid* g = new Grid();
  grid_build(cam, n_cur, cur_kps, *g);
  for (int i = 0; i < n_cur; i++) cur_match[i] = cur_preassigned ? cur_preassigned[i] : -1;
  int nmatches = 0;
  const bool bFactor = th != 1.0;
  std::vector<int> cand;
  for (int iMP = 0; iMP < n_mp; iMP++) {
    if (!in_view[iMP]) continue;  // mbTrackInView == false
    // Q13: PredictScale is unclamped in the reference; clamp to the pyramid.
    const int nPredictedLevel = std::min(std::max(pred_level[iMP], 0), nlevels - 1);
    float r = view_cos[iMP] > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos :131-137
    if (bFactor) r *= th;
    features_in_area(*g, cur_kps, proj_xy[2 * iMP], proj_xy[2 * iMP + 1],
                     r * scale_factors[nPredictedLevel], nPredictedLevel - 1, nPredictedLevel, cand);
    if (cand.empty()) continue;
    const uint8_t* d = mp_desc + 32 * (size_t)iMP;
    int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
    for (int idx : cand) {
      if (cur_match[idx] >= 0) continue;
      const int dist = descriptor_distance(d, cur_desc + 32 * (size_t)idx);
      if (dist < bestDist) {
        bestDist2 = bestDist;
        bestDist = dist;
        bestLevel2 = bestLevel;
        bestLevel = cur_kps[idx].octave;
        bestIdx = idx;
      } else if (dist < bestDist2) {
        bestLevel2 = cur_kps[idx].octave;
        bestDist2 = dist;
      }
    }
    if (bestDist <= TH_HIGH) {
      if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
      cur_match[bestIdx] = iMP;
      nmatches++;
    }
  }
  (void)cam;
  delete g;
  return nmatches;
}

// ORBmatcher::SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, th, ORBdist),
// ORBmatcher.cc:1472-1599 (relocalisation; Tracking.cc:2295,2309).
// kf_mp_valid[i]: vpMPs[i] && !isBad() && !sAlreadyFound.count(pMP).
// kf_mp_min_dist / kf_mp_max_dist: mfMinDistance / mfMaxDistance (MapPoint.cc:365-383).
// cur_preassigned[i2] >= 0 marks CurrentFrame.mvpMapPoints[i2] already set.
int orc_search_by_projection_keyframe(const orc_camera* cam, const float* Tcw, float th,
                                      int orb_dist, int check_ori, int n_kf,
                                      const orc_keypoint* kf_kps, const uint8_t* kf_mp_valid,
                                      const float* kf_mp_pos, const uint8_t* kf_mp_desc,
                                      const float* kf_mp_min_dist, const float* kf_mp_max_dist,
                                      float log_scale_factor, int n_cur,
                                      const orc_keypoint* cur_kps, const uint8_t* cur_desc,
                                      const int32_t* cur_preassigned, int nlevels,
                                      const float* scale_factors, int32_t* cur_match) {
  Grid* g = new Grid();
  grid_build(cam, n_cur, cur_kps, *g);
  for (int i = 0; i < n_cur; i++) cur_match[i] = cur_preassigned ? cur_preassigned[i] : -1;
  // Ow = -Rcw.t()*tcw (:1478): transposed gemm operand, double accumulation
  float Ow[3];
  for (int c = 0; c < 3; c++) {
    double s = (double)Tcw[c] * Tcw[3];
    s += (double)Tcw[4 + c] * Tcw[7];
    s += (double)Tcw[8 + c] * Tcw[11];
    Ow[c] = (float)(s * -1.0);
  }
  int nmatches = 0;
  std::vector<int> rotHist[HISTO_LENGTH];
  std::vector<int> cand;
  for (int i = 0; i < n_kf; i++) {
    if (!kf_mp_valid[i]) continue;
    const float* P = kf_mp_pos + 3 * i;
    float x3Dc[3];
    transform_point(Tcw, P, x3Dc);
    const float xc = x3Dc[0], yc = x3Dc[1];
    const float invzc = (float)(1.0 / x3Dc[2]);  // no depth test here (:1501-1506)
    const float u = cam->fx * xc * invzc + cam->cx;
    const float v = cam->fy * yc * invzc + cam->cy;
    if (u < g->minX || u > g->maxX) continue;
    if (v < g->minY || v > g->maxY) continue;
    const float PO[3] = {P[0] - Ow[0], P[1] - Ow[1], P[2] - Ow[2]};
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)PO[k] * PO[k];
    const float dist3D = (float)std::sqrt(s);  // cv::norm
    const float maxDistance = 1.2f * kf_mp_max_dist[i];
    const float minDistance = 0.8f * kf_mp_min_dist[i];
    if (dist3D < minDistance || dist3D > maxDistance) continue;
    // PredictScale (MapPoint.cc:385-394); Q13 clamp to the pyramid
    const float ratio = kf_mp_max_dist[i] / dist3D;
    int lvl = (int)std::ceil((float)std::log((double)ratio) / log_scale_factor);
    lvl = std::min(std::max(lvl, 0), nlevels - 1);
    const float radius = th * scale_factors[lvl];
    features_in_area(*g, cur_kps, u, v, radius, lvl - 1, lvl + 1, cand);
    if (cand.empty()) continue;
    const uint8_t* dMP = kf_mp_desc + 32 * (size_t)i;
    int bestDist = 256, bestIdx2 = -1;
    for (int i2 : cand) {
      if (cur_match[i2] >= 0) continue;
      const int dist = descriptor_distance(dMP, cur_desc + 32 * (size_t)i2);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx2 = i2;
      }
    }
    if (bestDist <= orb_dist) {
      cur_match[bestIdx2] = i;
      nmatches++;
      if (check_ori) rotHist[rot_bin(kf_kps[i].angle, cur_kps[bestIdx2].angle)].push_back(bestIdx2);
    }
  }
  if (check_ori) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
    for (int i = 0; i < HISTO_LENGTH; i++) {
      if (i != ind1 && i != ind2 && i != ind3) {
        for (int idx : rotHist[i]) {
          cur_match[idx] = -1;
          nmatches--;
        }
      }
    }
  }
  delete g;
  return nmatches;
}

// ORBmatcher::SearchForInitialization, :405-520
int orc_search_for_initialization(const orc_camera* cam, float nnratio, int check_ori, int n1,
                                  const orc_keypoint* kps1, const uint8_t* desc1, int n2,
                                  const orc_keypoint* kps2, const uint8_t* desc2,
                                  float* prev_matched_xy, int window, int32_t* matches12) {
  Grid* g = new Grid();
  grid_build(cam, n2, kps2, *g);
  int nmatches = 0;
  for (int i = 0; i < n1; i++) matches12[i] = -1;
  std::vector<int> rotHist[HISTO_LENGTH];
  std::vector<int> vMatchedDistance(n2, INT_MAX), vnMatches21(n2, -1);
  std::vector<int> cand;
  for (int i1 = 0; i1 < n1; i1++) {
    int level1 = kps1[i1].octave;
    if (level1 > 0) continue;
    features_in_area(*g, kps2, prev_matched_xy[2 * i1], prev_matched_xy[2 * i1 + 1], (float)window,
                     level1, level1, cand);
    if (cand.empty()) continue;
    const uint8_t* d1 = desc1 + 32 * (size_t)i1;
    int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
    for (int i2 : cand) {
      int dist = descriptor_distance(d1, desc2 + 32 * (size_t)i2);
      if (vMatchedDistance[i2] <= dist) continue;
      if (dist < bestDist) {
        bestDist2 = bestDist;
        bestDist = dist;
        bestIdx2 = i2;
      } else if (dist < bestDist2) {
        bestDist2 = dist;
      }
    }
    if (bestDist <= TH_LOW) {
      if (bestDist < (float)bestDist2 * nnratio) {
        if (vnMatches21[bestIdx2] >= 0) {
          matches12[vnMatches21[bestIdx2]] = -1;
          nmatches--;
        }
        matches12[i1] = bestIdx2;
        vnMatches21[bestIdx2] = i1;
        vMatchedDistance[bestIdx2] = bestDist;
        nmatches++;
        if (check_ori) rotHist[rot_bin(kps1[i1].angle, kps2[bestIdx2].angle)].push_back(i1);
      }
    }
  }
  if (check_ori) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
    for (int i = 0; i < HISTO_LENGTH; i++) {
      if (i == ind1 || i == ind2 || i == ind3) continue;
      for (int idx1 : rotHist[i]) {
        if (matches12[idx1] >= 0) {
          matches12[idx1] = -1;
          nmatches--;
        }
      }
    }
  }
  for (int i1 = 0; i1 < n1; i1++)
    if (matches12[i1] >= 0) {
      prev_matched_xy[2 * i1] = kps2[matches12[i1]].x;
      prev_matched_xy[2 * i1 + 1] = kps2[matches12[i1]].y;
    }
  delete g;
  return nmatches;
}

}  // extern "C"
