/*
 * assoc_ref.cpp -- CPU restatement of the EAO object association
 * (TEST INFRASTRUCTURE ONLY).
 *
 * Reference: src/Object.cc (whole), src/Converter.cc:194-212,
 * src/Tracking.cc:1241-1696 (object section of TrackWithMotionModel),
 * :2434-2468 (AssociateObjAndPoints), :2531-2598 (InitObjMap),
 * src/LocalMapping.cc:772-882 (object maintenance), include/isolation_forest.h.
 *
 * The replay is the deterministic single-threaded harness of SURVEY.md
 * appendix B: one call per frame with the pose, the YOLO boxes (file order,
 * score 0 -- Q1) and the tracked map points in keypoint-index order;
 * LocalMapping object maintenance runs when the caller says a keyframe was
 * inserted. Defined behaviour for reference UB: Q4 (int32 wraparound), Q7
 * (out_point = false), Q8 (erase stops after the last outlier), merge of a
 * one-frame object (Q29). Object lines (Tracking.cc:2472-2527,
 * AssociateObjAndLines + merge_break_lines) and yaw sampling (E14,
 * Tracking.cc:2602-2871) run for every flag but None / iForest; the frame's
 * line segments (Frame::all_lines_eigen) are a replay input.
 */
#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "iforest_ref.h"
#include "oracle.h"

namespace orc {

static const float kTTable[122][9] = {
#include "../eao-slam_amd/csrc/t_table.inc"
};

struct Rect {
  int x = 0, y = 0, w = 0, h = 0;
  Rect() {}
  Rect(int x_, int y_, int w_, int h_) : x(x_), y(y_), w(w_), h(h_) {}
  int area() const { return w * h; }
  // Rect_::contains(Point) after Point2f -> Point via cvRound (Q11)
  bool contains(float u, float v) const {
    int px = (int)std::lrintf(u), py = (int)std::lrintf(v);
    return x <= px && px < x + w && y <= py && py < y + h;
  }
};
static inline Rect rect_from_floats(float x, float y, float w, float h) {
  return Rect((int)x, (int)y, (int)w, (int)h);  // implicit float->int truncation (Q11)
}
static inline Rect rect_and(const Rect& a, const Rect& b) {
  int x1 = std::max(a.x, b.x), y1 = std::max(a.y, b.y);
  int w = std::min(a.x + a.w, b.x + b.w) - x1;
  int h = std::min(a.y + a.h, b.y + b.h) - y1;
  if (w <= 0 || h <= 0) return Rect();
  return Rect(x1, y1, w, h);
}
// Converter::bboxOverlapratio{,Former,Latter}, Converter.cc:194-212
static inline float iou(const Rect& a, const Rect& b) {
  int ov = rect_and(a, b).area();
  return (float)ov / ((float)(a.area() + b.area() - ov));
}
static inline float former(const Rect& a, const Rect& b) {
  int ov = rect_and(a, b).area();
  return (float)ov / ((float)(a.area()));
}
static inline float latter(const Rect& a, const Rect& b) {
  int ov = rect_and(a, b).area();
  return (float)ov / ((float)(b.area()));
}

static inline void transform_point(const float* T, const float* P, float* out) {
  for (int r = 0; r < 3; r++) {
    float t = T[4 * r] * P[0] + T[4 * r + 1] * P[1] + T[4 * r + 2] * P[2];
    out[r] = (float)((double)t + (double)T[4 * r + 3]);
  }
}

struct Cam {
  float fx, fy, cx, cy;
  int cols, rows;
};

// the projection used across Object.cc: invzc = 1.0/z (double->float),
// u = fx*xc*invzc + cx (float)
static inline void project(const Cam& c, const float* T, const float* P, float& u, float& v) {
  float pc[3];
  transform_point(T, P, pc);
  const float invzc = (float)(1.0 / pc[2]);
  u = c.fx * pc[0] * invzc + c.cx;
  v = c.fy * pc[1] * invzc + c.cy;
}


// ---------------------------------------------------------------- object lines
// Tracking::AssociateObjAndLines (Tracking.cc:2472-2527) and the cuboid utilities it
// calls: check_inside_box / align_left_right_edges (detect_3d_cuboid/object_3d_util.cpp:176-194),
// merge_break_lines (:349-436), fast_RemoveRow (matrix_utils.cpp:201-205).
static inline double norm2(double x, double y) { return std::sqrt(x * x + y * y); }

static void merge_break_lines(std::vector<double>& L, double dist_th, double angle_deg, double len_th) {
  int total = (int)L.size() / 4;
  int counter = 0;
  bool can = true;
  const double ath = angle_deg / 180.0 * M_PI;
  std::vector<double> ang;
  while (can && counter < 500) {
    counter++;
    can = false;
    ang.assign(total, 0.0);
    for (int i = 0; i < total; i++) ang[i] = std::atan2(L[4 * i + 3] - L[4 * i + 1], L[4 * i + 2] - L[4 * i]);
    for (int s1 = 0; s1 < total - 1; s1++) {
      for (int s2 = s1 + 1; s2 < total; s2++) {
        const double diff = std::abs(ang[s1] - ang[s2]);
        if (std::min(diff, M_PI - diff) < ath) {
          const double d12 = norm2(L[4 * s1 + 2] - L[4 * s2], L[4 * s1 + 3] - L[4 * s2 + 1]);
          const double d21 = norm2(L[4 * s2 + 2] - L[4 * s1], L[4 * s2 + 3] - L[4 * s1 + 1]);
          if (d12 < dist_th || d21 < dist_th) {
            const int a = L[4 * s1] < L[4 * s2] ? s1 : s2;
            const int b = L[4 * s1 + 2] > L[4 * s2 + 2] ? s1 : s2;
            const double st[2] = {L[4 * a], L[4 * a + 1]}, en[2] = {L[4 * b + 2], L[4 * b + 3]};
            const double ma = std::atan2(en[1] - st[1], en[0] - st[0]);
            const double t = std::abs(ang[s1] - ma);
            if (std::min(t, M_PI - t) < ath) {
              L[4 * s1] = st[0];
              L[4 * s1 + 1] = st[1];
              L[4 * s1 + 2] = en[0];
              L[4 * s1 + 3] = en[1];
              for (int c = 0; c < 4; c++) L[4 * s2 + c] = L[4 * (total - 1) + c];
              total--;
              can = true;
              break;
            }
          }
        }
      }
      if (can) break;
    }
  }
  std::vector<double> out;
  for (int i = 0; i < total; i++) {
    if (len_th > 0 && !(norm2(L[4 * i + 2] - L[4 * i], L[4 * i + 3] - L[4 * i + 1]) > len_th)) continue;
    for (int c = 0; c < 4; c++) out.push_back(L[4 * i + c]);
  }
  L.swap(out);
}

// ---------------------------------------------------------------- NP test
// Object_2D::NoParaDataAssociation, Object.cc:714-930
struct NPResult {
  int verdict, m, n;
  float w[3], r1, r2, gt[3], lt[3], eq[3];
};

static NPResult np_test(const std::vector<const float*>& frame_valid, int n_total,
                        const std::vector<const float*>& obj_valid) {
  NPResult R;
  std::memset(&R, 0, sizeof(R));
  int m = (int)frame_valid.size();
  int n = (int)obj_valid.size();
  R.m = m;
  R.n = n;
  if (m < 20) {
    R.verdict = 0;
    return R;
  }
  if (n < 20) {
    R.verdict = 2;
    return R;
  }
  std::vector<float> xs, ys, zs;
  if (n > 3 * m) {
    n = 3 * m;
    int step = n_total / n;
    std::vector<float> x, y, z;
    for (const float* p : obj_valid) {
      x.push_back(p[0]);
      y.push_back(p[1]);
      z.push_back(p[2]);
    }
    std::sort(x.begin(), x.end());
    std::sort(y.begin(), y.end());
    std::sort(z.begin(), z.end());
    for (size_t i = 0; i < x.size(); i += step) {
      xs.push_back(x[i]);
      ys.push_back(y[i]);
      zs.push_back(z[i]);
    }
    n = (int)xs.size();
  } else {
    for (const float* p : obj_valid) {
      xs.push_back(p[0]);
      ys.push_back(p[1]);
      zs.push_back(p[2]);
    }
    n = (int)xs.size();
  }
  R.n = n;
  float c12[3] = {0, 0, 0}, c21[3] = {0, 0, 0}, c00[3] = {0, 0, 0};
  const std::vector<float>* S[3] = {&xs, &ys, &zs};
  for (const float* p : frame_valid) {
    for (int a = 0; a < 3; a++) {
      double v1 = p[a];
      for (float s : *S[a]) {
        double v2 = s;
        if (v1 > v2) c12[a]++;
        else if (v1 < v2) c21[a]++;
        else if (v1 == v2) c00[a]++;
      }
    }
  }
  // Q4: int products wrap (defined as int32 two's complement)
  int mm = (int)((uint32_t)m * (uint32_t)(m + 1) / 2u);
  int nn = (int)((uint32_t)n * (uint32_t)(n + 1) / 2u);
  for (int a = 0; a < 3; a++) {
    R.w[a] = std::min(c12[a] + mm, c21[a] + nn) + c00[a] / 2;
    R.gt[a] = c12[a];
    R.lt[a] = c21[a];
    R.eq[a] = c00[a];
  }
  int prod = (int)((uint32_t)m * (uint32_t)n * (uint32_t)(m + n + 1));
  int q = prod / 12;
  R.r1 = (float)(0.5 * m * (m + n + 1) - 1.282 * std::sqrt((double)q));
  R.r2 = (float)(0.5 * m * (m + n + 1) + 1.282 * std::sqrt((double)q));
  int add = 0;
  for (int a = 0; a < 3; a++)
    if (R.w[a] > R.r1 && R.w[a] < R.r2) add++;
  R.verdict = (add == 3) ? 1 : 2;
  return R;
}

// ---------------------------------------------------------------- replay model
struct MapPoint {
  int id;
  float pos[3];
  bool bad = false;
  bool out_point = false;  // Q7
  float feat_u = 0, feat_v = 0;
  std::map<int, int> object_id_vector;
  int object_id = -1, object_class = -1;
};

struct ObjMap;
struct Obj2D {
  int class_id = -1;
  float score = 0.f;
  int bx = 0, by = 0, bw = 0, bh = 0;  // BoxSE (cv::Rect)
  Rect box;
  Rect feat_rect;
  std::vector<MapPoint*> pts;
  float sum[3] = {0, 0, 0};
  float pos[3] = {0, 0, 0};
  float std_[3] = {0, 0, 0};
  bool bad = false, few = false, on_edge = false, current = false;
  int mnId = -1, which_time = 0;
  int method = 0;  // replay output: how it was associated
  int input_index = -1;
  std::vector<double> lines;  // mObjLinesEigen (rows x1, y1, x2, y2), Tracking.cc:2524
  // cv::Mat aliasing (Object.cc:677, Tracking.cc:2563): the detection that
  // creates a map object shares its _Pos buffer with that object's mCenter3D,
  // which ComputeMeanAndStandard later rewrites in place (Object.cc:995).
  struct ObjMap* alias = nullptr;
};

struct Cuboid {
  double corner[8][3] = {};
  double corner_w[8][3] = {};
  float x_min = 0, x_max = 0, y_min = 0, y_max = 0, z_min = 0, z_max = 0;
  double center[3] = {0, 0, 0};
  float lenth = 0, width = 0, height = 0;
  double q[4] = {1, 0, 0, 0};      // pose rotation (w,x,y,z)
  double t[3] = {0, 0, 0};         // pose translation
  double qn[4] = {1, 0, 0, 0};     // pose_without_yaw
  double tn[3] = {0, 0, 0};
  float rotY = 0, rotP = 0, rotR = 0;
  float rmax = 0;
  float err_parallel = 0, err_yaw = 0;  // mfErrorParallel, mfErroeYaw
};

struct ObjMap {
  std::vector<Obj2D*> frames;
  Rect last, lastlast, proj;
  int mnId = 0, mnClass = 0, confidence = 0;
  bool first_observe = false;
  int added = 0, last_add = 0, lastlast_add = 0;
  std::vector<MapPoint*> pts;
  float sum[3] = {0, 0, 0};
  float center[3] = {0, 0, 0};
  float std_[3] = {0, 0, 0};
  float cstd[3] = {0, 0, 0};
  float cstd_all = 0;
  std::map<int, int> reobj, sametime;
  bool bad = false;
  Cuboid cub;
  std::vector<std::array<float, 5>> angles;  // mvAngleTimesAndScore (Vector5f rows)
};

static inline const float* fpos(const Obj2D* f) { return f->alias ? f->alias->center : f->pos; }

// --- minimal Eigen/g2o SE3Quat restatement (Eigen 3.2 Quaternion, g2o se3quat.h)
static void quat_from_R(const double R[3][3], double q[4]) {
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
    int j = (i + 1) % 3, k = (j + 1) % 3;
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
  // SE3Quat::normalizeRotation
  if (q[0] < 0)
    for (int a = 0; a < 4; a++) q[a] = -q[a];
  double nrm = std::sqrt(((q[1] * q[1] + q[3] * q[3]) + (q[2] * q[2] + q[0] * q[0])));
  for (int a = 0; a < 4; a++) q[a] = q[a] / nrm;
}
static void quat_rotate(const double q[4], const double v[3], double out[3]) {
  // Eigen _transformVector: uv = vec x v; uv += uv; v + w*uv + vec x uv
  const double x = q[1], y = q[2], z = q[3], w = q[0];
  double uv[3] = {y * v[2] - z * v[1], z * v[0] - x * v[2], x * v[1] - y * v[0]};
  for (int a = 0; a < 3; a++) uv[a] += uv[a];
  double c2[3] = {y * uv[2] - z * uv[1], z * uv[0] - x * uv[2], x * uv[1] - y * uv[0]};
  for (int a = 0; a < 3; a++) out[a] = v[a] + w * uv[a] + c2[a];
}
static void pose_apply(const double q[4], const double t[3], const double v[3], double out[3]) {
  double r[3];
  quat_rotate(q, v, r);
  for (int a = 0; a < 3; a++) out[a] = r[a] + t[a];
}
static void pose_inverse_apply(const double q[4], const double t[3], const double v[3], double out[3]) {
  double qc[4] = {q[0], -q[1], -q[2], -q[3]};
  double mt[3] = {t[0] * -1., t[1] * -1., t[2] * -1.};
  double ti[3];
  quat_rotate(qc, mt, ti);
  pose_apply(qc, ti, v, out);
}

static inline const float* fpos(const Obj2D* f);

class Replay {
 public:
  std::string flag;
  Cam cam;
  bool biForest = true;  // Object.cc:31 (sticky, Q6)
  std::vector<ObjMap*> objs;
  std::map<int, MapPoint*> mps;
  std::vector<Obj2D*> all2d;  // ownership
  bool ini = false;
  long ini_frame = 0;
  unsigned long cur_id = 0;
  float T[16];

  ~Replay() {
    for (auto* o : objs) delete o;
    for (auto& kv : mps) delete kv.second;
    for (auto* o : all2d) delete o;
  }

  bool is(const char* f) const { return flag == f; }

  // frame line sets staged by orc_replay_lines, consumed one per frame
  std::vector<std::vector<float>> staged_lines;
  size_t staged_next = 0;

  // Tracking::AssociateObjAndLines, Tracking.cc:2472-2527
  void associate_lines(const std::vector<Obj2D*>& o2, const std::vector<float>& fl) {
    std::vector<double> all(fl.begin(), fl.end());  // all_lines_eigen (float Mat -> double)
    const int n = (int)all.size() / 4;
    for (int i = 0; i < n; i++)  // align_left_right_edges
      if (all[4 * i + 2] < all[4 * i]) {
        std::swap(all[4 * i], all[4 * i + 2]);
        std::swap(all[4 * i + 1], all[4 * i + 3]);
      }
    for (auto* f : o2) {
      const double l = std::max(0.0, f->bx - 15.0);
      const double r = (double)std::min(cam.cols, f->bx + f->bw + 15);
      const double t = std::max(0.0, f->by - 15.0);
      const double b = (double)std::min(cam.rows, f->by + f->bh + 15);
      std::vector<double> in;
      for (int i = 0; i < n; i++) {
        const double* e = &all[4 * i];
        if (l <= e[0] && e[0] <= r && t <= e[1] && e[1] <= b && l <= e[2] && e[2] <= r && t <= e[3] &&
            e[3] <= b)
          in.insert(in.end(), e, e + 4);
      }
      merge_break_lines(in, 20, 5, 30);
      f->lines.swap(in);
    }
  }

  // Tracking::SampleObjYaw (Tracking.cc:2624-2871) with WorldToImg (:2602-2620)
  void sample_yaw(ObjMap* o) {
    if (flag == "None" || flag == "iForest") return;
    const std::vector<double>& L = o->frames.back()->lines;
    const int nAll = (int)L.size() / 4;
    int numMax = 0;
    float fError = 0.0f, fErrorYaw = 0.0f, sampleYaw = 0.0f;
    Cuboid& c = o->cub;
    float ctr[3], rel[8][3];
    for (int a = 0; a < 3; a++) ctr[a] = (float)c.center[a];
    for (int k = 0; k < 8; k++)
      for (int a = 0; a < 3; a++) rel[k][a] = (float)c.corner_w[k][a] - ctr[a];
    for (int i = 0; i < 30; i++) {
      const float roll = 0.0f, pitch = 0.0f;
      const float yaw = i < 15 ? (float)((0.0 - i * 3.0) / 180.0 * M_PI) : (float)((0.0 + (i - 15) * 3.0) / 180.0 * M_PI);
      float error = 0.0f, errorYaw = 0.0f;
      const float cp = std::cos(pitch), sp = std::sin(pitch), sr = std::sin(roll), cr = std::cos(roll);
      const float sy = (float)std::sin((double)yaw), cy = (float)std::cos((double)yaw);  // Q26
      const float R[3][3] = {{cp * cy, (sr * sp * cy) - (cr * sy), (cr * sp * cy) + (sr * sy)},
                             {cp * sy, (sr * sp * sy) + (cr * cy), (cr * sp * sy) - (sr * cy)},
                             {-sp, sr * cp, cr * cp}};
      float px[8], py[8];
      for (int k = 0; k < 8; k++) {
        float w[3];
        for (int r = 0; r < 3; r++) {  // Ryaw * corner + center: cv::Mat gemm (Q12)
          const float d = R[r][0] * rel[k][0] + R[r][1] * rel[k][1] + R[r][2] * rel[k][2];
          w[r] = (float)((double)d + (double)ctr[r]);
        }
        project(cam, T, w, px[k], py[k]);  // WorldToImg
      }
      auto edge = [&](int a, int b, float& ang, float& len) {  // point_b vs point_a, left -> right
        if (px[b] > px[a])
          ang = std::atan2(py[b] - py[a], px[b] - px[a]);
        else
          ang = std::atan2(py[a] - py[b], px[a] - px[b]);
        len = std::sqrt((py[b] - py[a]) * (py[b] - py[a]) + (px[b] - px[a]) * (px[b] - px[a]));
      };
      float angle1, angle2, angle3, l1, l2, l3;
      edge(4, 5, angle1, l1);  // point5 -> point6
      edge(5, 6, angle2, l2);  // point6 -> point7
      edge(1, 5, angle3, l3);  // point2 -> point6
      int num = 0;
      for (int li = 0; li < nAll; li++) {
        const double x1 = L[4 * li], y1 = L[4 * li + 1], x2 = L[4 * li + 2], y2 = L[4 * li + 3];
        const float angle = (float)std::atan2(y2 - y1, x2 - x1);
        const float d1 = (float)std::abs((double)(angle * 180) / M_PI - (double)(angle1 * 180) / M_PI);
        const float d2 = (float)std::abs((double)(angle * 180) / M_PI - (double)(angle2 * 180) / M_PI);
        const float d3 = (float)std::abs((double)(angle * 180) / M_PI - (double)(angle3 * 180) / M_PI);
        const float th = 5.0f;
        if (o->mnClass == 56) {
          if ((d2 < th) || (d3 < th)) num++;
          if (d1 < th) num += 3;
        } else {
          const float mn = std::min(std::min(l1, l2), l3);
          if (mn == l1) {
            if ((d2 < th) || (d3 < th)) {
              num++;
              if (d2 < th) error += d2;
              if (d3 < th) error += d3;
            }
            errorYaw += std::min(d2, d3);
          }
          if (mn == l2) {
            if ((d1 < th) || (d3 < th)) {
              num++;
              if (d1 < th) error += d1;
              if (d3 < th) error += d3;
            }
            errorYaw += std::min(d3, d1);
          }
          if (mn == l3) {
            if ((d1 < th) || (d2 < th)) {
              num++;
              if (d1 < th) error += d1;
              if (d2 < th) error += d2;
            }
            errorYaw += std::min(d2, d1);
          }
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
    // std::sort with VIC (index = 1, Tracking.cc:63-68): the same libstdc++ introsort
    std::sort(o->angles.begin(), o->angles.end(),
              [](const std::array<float, 5>& l, const std::array<float, 5>& r) { return l[1] > r[1]; });
    int best = 0;
    float best_score = 0;
    for (int i = 0; i < std::min(3, (int)o->angles.size()); i++) {
      const float f = o->angles[i][2];
      if (f >= best_score) {
        best_score = f;
        best = i;
      }
    }
    c.rotY = o->angles[best][0];
    c.err_parallel = o->angles[best][3];
    c.err_yaw = o->angles[best][4];
  }

  // Object_Map::UpdateObjPose, Object.cc:2193-2248
  void update_pose(ObjMap* o) {
    Cuboid& c = o->cub;
    float cp = std::cos(c.rotP), sp = std::sin(c.rotP), sr = std::sin(c.rotR), cr = std::cos(c.rotR);
    float sy = std::sin(c.rotY), cy = std::cos(c.rotY);
    float Rf[3][3] = {{cp * cy, (sr * sp * cy) - (cr * sy), (cr * sp * cy) + (sr * sy)},
                      {cp * sy, (sr * sp * sy) + (cr * cy), (cr * sp * sy) - (sr * cy)},
                      {-sp, sr * cp, cr * cp}};
    double R[3][3];
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) R[a][b] = (double)Rf[a][b];  // via Twobj (CV_32F)
    quat_from_R(R, c.q);
    for (int a = 0; a < 3; a++) c.t[a] = (double)(float)c.center[a];
    double I[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    quat_from_R(I, c.qn);
    c.tn[0] = (double)o->center[0];
    c.tn[1] = (double)(float)c.center[1];
    c.tn[2] = (double)o->center[2];
  }

  // Object_Map::ComputeMeanAndStandard, Object.cc:967-1198
  void mean_and_standard(ObjMap* o) {
    for (int a = 0; a < 3; a++) o->sum[a] = 0;
    for (auto it = o->pts.begin(); it != o->pts.end();) {
      if ((*it)->bad)
        it = o->pts.erase(it);
      else {
        for (int a = 0; a < 3; a++) o->sum[a] += (*it)->pos[a];
        ++it;
      }
    }
    const size_t np = o->pts.size();
    const float sc = (float)(1. / (double)np);
    for (int a = 0; a < 3; a++) o->center[a] = o->sum[a] * sc + 0.0f;
    float s2[3] = {0, 0, 0};
    std::vector<float> xp, yp, zp;
    for (auto* p : o->pts) {
      for (int a = 0; a < 3; a++) s2[a] += (p->pos[a] - o->center[a]) * (p->pos[a] - o->center[a]);
      xp.push_back(p->pos[0]);
      yp.push_back(p->pos[1]);
      zp.push_back(p->pos[2]);
    }
    for (int a = 0; a < 3; a++) o->std_[a] = std::sqrt(s2[a] / (float)np);
    if (xp.empty()) return;
    float c2[3] = {0, 0, 0};
    for (auto* f : o->frames) {
      const float* fp = fpos(f);
      for (int a = 0; a < 3; a++) c2[a] += (fp[a] - o->center[a]) * (fp[a] - o->center[a]);
    }
    for (int a = 0; a < 3; a++) o->cstd[a] = std::sqrt(c2[a] / (float)o->frames.size());
    Cuboid& c = o->cub;
    if (o->frames.size() < 5) {
      std::sort(xp.begin(), xp.end());
      std::sort(yp.begin(), yp.end());
      std::sort(zp.begin(), zp.end());
      float x_min = xp[0], x_max = xp.back(), y_min = yp[0], y_max = yp.back(), z_min = zp[0],
            z_max = zp.back();
      c.center[0] = (x_max + x_min) / 2;
      c.center[1] = (y_max + y_min) / 2;
      c.center[2] = (z_max + z_min) / 2;
      c.x_min = x_min; c.x_max = x_max;
      c.y_min = y_min; c.y_max = y_max;
      c.z_min = z_min; c.z_max = z_max;
      c.lenth = x_max - x_min;
      c.width = y_max - y_min;
      c.height = z_max - z_min;
      const float X[2] = {x_min, x_max}, Y[2] = {y_min, y_max}, Z[2] = {z_min, z_max};
      static const int cx[8] = {0, 1, 1, 0, 0, 1, 1, 0}, cy[8] = {0, 0, 1, 1, 0, 0, 1, 1},
                       cz[8] = {0, 0, 0, 0, 1, 1, 1, 1};
      for (int k = 0; k < 8; k++) {
        c.corner[k][0] = c.corner_w[k][0] = X[cx[k]];
        c.corner[k][1] = c.corner_w[k][1] = Y[cy[k]];
        c.corner[k][2] = c.corner_w[k][2] = Z[cz[k]];
      }
    }
    update_pose(o);
    std::vector<float> xo, yo, zo;
    for (auto* p : o->pts) {
      double v[3] = {p->pos[0], p->pos[1], p->pos[2]}, r[3];
      pose_inverse_apply(c.q, c.t, v, r);
      xo.push_back((float)r[0]);
      yo.push_back((float)r[1]);
      zo.push_back((float)r[2]);
    }
    if (xo.empty()) return;
    std::sort(xo.begin(), xo.end());
    std::sort(yo.begin(), yo.end());
    std::sort(zo.begin(), zo.end());
    const float X[2] = {xo[0], xo.back()}, Y[2] = {yo[0], yo.back()}, Z[2] = {zo[0], zo.back()};
    static const int cx[8] = {0, 1, 1, 0, 0, 1, 1, 0}, cy[8] = {0, 0, 1, 1, 0, 0, 1, 1},
                     cz[8] = {0, 0, 0, 0, 1, 1, 1, 1};
    for (int k = 0; k < 8; k++) {
      double v[3] = {X[cx[k]], Y[cy[k]], Z[cz[k]]};
      pose_apply(c.q, c.t, v, c.corner[k]);
      pose_apply(c.qn, c.tn, v, c.corner_w[k]);
    }
    c.lenth = X[1] - X[0];
    c.width = Y[1] - Y[0];
    c.height = Z[1] - Z[0];
    for (int a = 0; a < 3; a++) c.center[a] = (c.corner[1][a] + c.corner[7][a]) / 2;
    update_pose(o);
    float fRMax = 0.0f;
    for (int k = 0; k < 8; k++) {
      float d[3];
      for (int a = 0; a < 3; a++) d[a] = o->center[a] - (float)c.corner[k][a];
      float tmp = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
      fRMax = std::max(fRMax, tmp);
    }
    c.rmax = fRMax;
    float dis = 0;
    for (auto* f : o->frames) {
      float e[3];
      const float* fp = fpos(f);
      for (int a = 0; a < 3; a++) e[a] = (fp[a] - o->center[a]) * (fp[a] - o->center[a]);
      dis += std::sqrt(e[0] + e[1] + e[2]);
    }
    o->cstd_all = std::sqrt(dis / (float)o->frames.size());
  }

  // Object_Map::IsolationForestDeleteOutliers, Object.cc:1202-1309
  void iforest_delete(ObjMap* o) {
    if (!biForest) return;
    if (o->mnClass == 75 || o->mnClass == 64 || o->mnClass == 65) return;
    float th = 0.6f;
    if (o->mnClass == 62) th = 0.65f;
    if (o->pts.size() < 30) return;
    std::vector<float> data;
    for (auto* p : o->pts)
      for (int a = 0; a < 3; a++) data.push_back(p->pos[a]);
    std::vector<double> scores;
    if (!iforest_scores(data.data(), (uint32_t)o->pts.size(), 50, 12345,
                        (uint32_t)((int)o->pts.size() / 2), scores))
      return;
    std::vector<int> outl;
    for (uint32_t i = 0; i < (uint32_t)o->pts.size(); i++)
      if (scores[i] > th) outl.push_back((int)i);
    if (outl.empty()) return;
    int num = -1, k = 0;
    for (auto it = o->pts.begin(); it != o->pts.end();) {
      num++;
      if (k < (int)outl.size() && num == outl[k]) {  // Q8
        k++;
        for (int a = 0; a < 3; a++) o->sum[a] -= (*it)->pos[a];
        it = o->pts.erase(it);
      } else
        ++it;
    }
  }

  // Object_Map::ComputeProjectRectFrame, Object.cc:1558-1603
  void project_rect(ObjMap* o) {
    std::vector<float> xs, ys;
    for (auto* p : o->pts) {
      float u, v;
      project(cam, T, p->pos, u, v);
      xs.push_back(u);
      ys.push_back(v);
    }
    if (xs.empty()) return;
    std::sort(xs.begin(), xs.end());
    std::sort(ys.begin(), ys.end());
    float x_min = xs[0], x_max = xs.back(), y_min = ys[0], y_max = ys.back();
    if (x_min < 0) x_min = 0;
    if (y_min < 0) y_min = 0;
    if (x_max > cam.cols) x_max = (float)cam.cols;
    if (y_max > cam.rows) y_max = (float)cam.rows;
    o->proj = rect_from_floats(x_min, y_min, x_max - x_min, y_max - y_min);
  }

  static bool same_pos(const MapPoint* a, const MapPoint* b) {
    return (a->pos[0] - b->pos[0]) == 0 && (a->pos[1] - b->pos[1]) == 0 && (a->pos[2] - b->pos[2]) == 0;
  }

  static void vote(MapPoint* p, int id) {
    auto it = p->object_id_vector.find(id);
    if (it != p->object_id_vector.end()) it->second += 1;
    else p->object_id_vector[id] = 1;
  }

  static void add_reobj(ObjMap* o, int id) {
    auto it = o->reobj.find(id);
    if (it != o->reobj.end()) it->second += 1;
    else o->reobj[id] = 1;
  }

  // Object_Map::DataAssociateUpdate, Object.cc:1313-1554
  bool update(ObjMap* o, Obj2D* f, int Flag) {
    if (f->class_id != o->mnClass) return false;
    if (Flag != 1 && Flag != 4) {
      project_rect(o);
      Rect r1 = o->proj;
      std::vector<float> xs, ys;
      for (auto* p : f->pts) {
        float u, v;
        project(cam, T, p->pos, u, v);
        xs.push_back(u);
        ys.push_back(v);
      }
      for (auto* p : o->pts) {
        float u, v;
        project(cam, T, p->pos, u, v);
        xs.push_back(u);
        ys.push_back(v);
      }
      std::sort(xs.begin(), xs.end());
      std::sort(ys.begin(), ys.end());
      float x_min = xs[0], x_max = xs.back(), y_min = ys[0], y_max = ys.back();
      if (x_min < 0) x_min = 0;
      if (y_min < 0) y_min = 0;
      if (x_max > cam.cols) x_max = (float)cam.cols;
      if (y_max > cam.rows) y_max = (float)cam.rows;
      Rect r2 = rect_from_floats(x_min, y_min, x_max - x_min, y_max - y_min);
      float fIou = iou(r1, r2);
      float fIou2 = former(r2, f->box);
      if ((fIou < 0.5) && (fIou2 < 0.8)) return false;
    }
    if (o->last_add != (int)cur_id) {
      o->lastlast_add = o->last_add;
      o->last_add = (int)cur_id;
      o->lastlast = o->last;
      o->last = f->box;
      o->confidence++;
      f->current = true;
      o->frames.push_back(f);
    } else
      return false;
    f->mnId = o->mnId;
    f->which_time = o->confidence;
    for (auto* p : f->pts) {
      float d[3];
      for (int a = 0; a < 3; a++) d[a] = o->center[a] - p->pos[a];
      float fDis = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
      float th = 1.0f;
      if (o->frames.size() > 5) th = 0.9f;
      if (fDis > th * o->cub.rmax) continue;
      if (o->frames.size() >= 10 && (o->mnClass == 56 || o->mnClass == 77)) {
        double v[3] = {p->pos[0], p->pos[1], p->pos[2]}, s[3];
        pose_inverse_apply(o->cub.q, o->cub.t, v, s);
        if (std::fabs(s[0]) > 1.2 * o->cub.lenth / 2 || std::fabs(s[1]) > 1.2 * o->cub.width / 2 ||
            std::fabs(s[2]) > 1.2 * o->cub.height / 2)
          continue;
      }
      p->object_id = o->mnId;
      p->object_class = o->mnClass;
      vote(p, p->object_id);
      bool new_point = true;
      for (auto* q : o->pts)
        if (same_pos(p, q)) {
          new_point = false;
          break;
        }
      if (new_point) {
        o->pts.push_back(p);
        for (int a = 0; a < 3; a++) o->sum[a] += p->pos[a];
      }
    }
    if (f->bx > 25 && f->by > 25 && f->bx + f->bw < cam.cols - 25 && f->by + f->bh < cam.rows - 25) {
      for (auto it = o->pts.begin(); it != o->pts.end();) {
        int votes = 0;
        auto vit = (*it)->object_id_vector.find(o->mnId);
        if (vit != (*it)->object_id_vector.end()) votes = vit->second;
        if (votes > 8) {
          ++it;
          continue;
        }
        float u, v;
        project(cam, T, (*it)->pos, u, v);
        if ((u > 0 && u < cam.cols) && (v > 0 && v < cam.rows)) {
          if (!f->box.contains(u, v)) {
            for (int a = 0; a < 3; a++) o->sum[a] -= (*it)->pos[a];
            it = o->pts.erase(it);
          } else
            ++it;
        } else
          ++it;
      }
    }
    mean_and_standard(o);
    iforest_delete(o);
    return true;
  }

  NPResult np_for(Obj2D* f, ObjMap* o) {
    std::vector<const float*> fv, ov;
    for (auto* p : f->pts)
      if (!(p->bad || p->out_point)) fv.push_back(p->pos);
    for (auto* p : o->pts)
      if (!(p->bad || p->out_point)) ov.push_back(p->pos);
    return np_test(fv, (int)o->pts.size(), ov);
  }

  // Object_2D::ObjectDataAssociation, Object.cc:162-710
  void associate(Obj2D* f) {
    if (flag == "None") biForest = false;
    const Rect RectCurrent = f->box;
    Rect RectPredict;
    float IouMax = 0;
    bool bAssoByIou = false;
    int nAssoByIouId = -1, IouMaxObjID = -1;
    float IouThreshold = 0.5;
    const int N = (int)objs.size();
    if (flag != "NA" && flag != "NP") {
      for (int i = 0; i < N; i++) {
        ObjMap* o = objs[i];
        if (f->class_id != o->mnClass) continue;
        if (o->bad) continue;
        if ((unsigned long)(long)o->last_add == cur_id - 1) {
          if ((unsigned long)(long)o->lastlast_add == cur_id - 2) {
            float ltx = (float)(o->last.x * 2 - o->lastlast.x);
            if (ltx < 0) ltx = 0;
            float lty = (float)(o->last.y * 2 - o->lastlast.y);
            if (lty < 0) lty = 0;
            float rdx = (float)((o->last.x + o->last.w) * 2 - (o->lastlast.x + o->lastlast.w));
            if (ltx > cam.cols) rdx = (float)cam.cols;
            float rdy = (float)((o->last.y + o->last.h) * 2 - (o->lastlast.y + o->lastlast.h));
            if (lty > cam.rows) rdy = (float)cam.rows;
            RectPredict = rect_from_floats(ltx, lty, rdx - ltx, rdy - lty);
            IouThreshold = 0.6f;
          } else
            RectPredict = o->last;
          float I = iou(RectCurrent, RectPredict);
          if ((I > IouThreshold) && I > IouMax) {
            IouMax = I;
            IouMaxObjID = i;
          }
        }
      }
      if (IouMax > 0 && IouMaxObjID >= 0) {
        if (update(objs[IouMaxObjID], f, 1)) {
          bAssoByIou = true;
          nAssoByIouId = IouMaxObjID;
          f->method = 1;
        }
      }
    }
    bool bAssoByNp = false;
    int nAssoByNPId = -1;
    std::vector<int> vNP;
    if (flag != "NA" && flag != "IoU") {
      for (int i = (int)objs.size() - 1; i >= 0; i--) {
        ObjMap* o = objs[i];
        if (f->class_id != o->mnClass) continue;
        if (o->bad) continue;
        NPResult R = np_for(f, o);
        np_log.push_back({f->input_index, o->mnId, R});
        if (R.verdict == 0) break;
        if (R.verdict == 2) continue;
        vNP.push_back(i);
      }
      if (vNP.size() >= 1) {
        if (bAssoByIou) {
          for (size_t i = 0; i < vNP.size(); i++) {
            if (vNP[i] == nAssoByIouId) continue;
            add_reobj(objs[nAssoByIouId], objs[vNP[i]]->mnId);
          }
        } else {
          for (size_t i = 0; i < vNP.size(); i++) {
            if (update(objs[vNP[i]], f, 2)) {
              bAssoByNp = true;
              nAssoByNPId = vNP[i];
              f->method = 2;
              if (vNP.size() > i + 1) {
                for (size_t j = i + 1; j < vNP.size(); j++) add_reobj(objs[vNP[i]], objs[vNP[j]]->mnId);
                break;
              }
            }
          }
        }
      }
    }
    bool bAssoByProject = false;
    int nAssoByProId = -1;
    std::vector<int> vPro;
    if (flag != "NA" && flag != "IoU" && flag != "NP") {
      float fIouMax = 0.0f;
      int ProIouMaxObjId = -1;
      for (int i = (int)objs.size() - 1; i >= 0; i--) {
        ObjMap* o = objs[i];
        if (f->class_id != o->mnClass) continue;
        if (o->bad) continue;
        int df = (int)o->frames.size();
        if (f->pts.size() >= 10 && df > 8) continue;
        float a = iou(RectCurrent, o->proj);
        float b = iou(f->feat_rect, o->proj);
        a = std::max(a, b);
        if (a >= 0.25 && a > fIouMax) {
          fIouMax = a;
          ProIouMaxObjId = i;
          vPro.push_back(i);
        }
      }
      if (fIouMax >= 0.25) {
        std::sort(vPro.begin(), vPro.end());
        if (bAssoByIou || bAssoByNp) {
          for (int j = (int)vPro.size() - 1; j >= 0; j--) {
            int ReId = -1;
            if (bAssoByIou) ReId = nAssoByIouId;
            if (bAssoByNp) ReId = nAssoByNPId;
            if (vPro[j] == ReId) continue;
            add_reobj(objs[ReId], objs[vPro[j]]->mnId);
          }
        } else {
          if (update(objs[ProIouMaxObjId], f, 4)) {
            bAssoByProject = true;
            nAssoByProId = ProIouMaxObjId;
            f->method = 4;
          }
          for (int j = (int)vPro.size() - 1; j >= 0; j--) {
            if (vPro[j] == ProIouMaxObjId) continue;
            add_reobj(objs[ProIouMaxObjId], objs[vPro[j]]->mnId);
          }
        }
      }
    }
    bool bAssoByT = false;
    std::vector<int> vT, vTL;
    if (flag != "NA" && flag != "IoU" && flag != "NP") {
      for (int i = (int)objs.size() - 1; i >= 0; i--) {
        ObjMap* o = objs[i];
        if (f->class_id != o->mnClass) continue;
        if (o->bad) continue;
        int df = (int)o->frames.size();
        if (df <= 8) continue;
        float a = iou(RectCurrent, o->proj);
        float b = iou(f->feat_rect, o->proj);
        a = std::max(a, b);
        float dx = std::fabs(o->center[0] - f->pos[0]);
        float dy = std::fabs(o->center[1] - f->pos[1]);
        float dz = std::fabs(o->center[2] - f->pos[2]);
        // sqrt(int) is the double overload: the quotient is evaluated in double
        float tx = (float)(dx / (o->cstd[0] / std::sqrt((double)df)));
        float ty = (float)(dy / (o->cstd[1] / std::sqrt((double)df)));
        float tz = (float)(dz / (o->cstd[2] / std::sqrt((double)df)));
        t_log.push_back({f->input_index, o->mnId, tx, ty, tz});
        const float* row = kTTable[std::min(df - 1, 121)];
        if (tx < row[5] && ty < row[5] && tz < row[5]) {
          vT.push_back(i);
        } else if (a > 0.25) {
          if (tx < row[8] && ty < row[8] && tz < row[8])
            vT.push_back(i);
          else if ((a > 0.25) && ((tx + ty + tz) / 3 < 10))
            vT.push_back(i);
          else
            vTL.push_back(i);
        } else if ((tx + ty + tz) / 3 < 4) {
          project_rect(o);
          float c = iou(RectCurrent, o->proj);
          float d = iou(f->feat_rect, o->proj);
          c = std::max(c, d);
          if (c > 0.25) vTL.push_back(i);
        }
      }
      if (bAssoByIou || bAssoByNp || bAssoByProject) {
        int ReId = -1;
        if (bAssoByIou) ReId = nAssoByIouId;
        if (bAssoByNp) ReId = nAssoByNPId;
        if (bAssoByProject) ReId = nAssoByProId;
        for (size_t j = 0; j < vT.size(); j++) {
          if (vT[j] == ReId) continue;
          add_reobj(objs[ReId], objs[vT[j]]->mnId);
        }
        for (size_t j = 0; j < vTL.size(); j++) {
          if (vTL[j] == ReId) continue;
          add_reobj(objs[ReId], objs[vTL[j]]->mnId);
        }
      } else {
        for (size_t i = 0; i < vT.size(); i++) {
          if (update(objs[vT[i]], f, 3)) {
            bAssoByT = true;
            int nAssoByTId = vT[i];
            f->method = 3;
            for (size_t j = i + 1; j < vT.size(); j++) add_reobj(objs[nAssoByTId], objs[vT[j]]->mnId);
            for (size_t j = 0; j < vTL.size(); j++) {
              if (vTL[j] == nAssoByTId) continue;
              add_reobj(objs[nAssoByTId], objs[vTL[j]]->mnId);
            }
            break;
          }
        }
      }
    }
    if (bAssoByIou || bAssoByNp || bAssoByProject || bAssoByT) return;
    if (f->bx < 10 || f->by < 10 || f->bx + f->bw > cam.cols - 10 || f->by + f->bh > cam.rows - 10) {
      f->bad = true;
      return;
    }
    ObjMap* o = new ObjMap();
    o->frames.push_back(f);
    o->mnId = (int)objs.size();
    o->mnClass = f->class_id;
    o->confidence = 1;
    o->first_observe = true;
    o->added = o->last_add = o->lastlast_add = (int)cur_id;
    o->last = f->box;
    for (int a = 0; a < 3; a++) {
      o->sum[a] = f->sum[a];
      o->center[a] = f->pos[a];
    }
    for (auto* p : f->pts) {
      p->object_id = o->mnId;
      p->object_class = o->mnClass;
      p->object_id_vector.insert(std::make_pair(o->mnId, 1));
      o->pts.push_back(p);
    }
    f->mnId = o->mnId;
    f->which_time = o->confidence;
    f->current = true;
    f->method = 5;
    f->alias = o;
    iforest_delete(o);
    mean_and_standard(o);
    objs.push_back(o);
  }

  // Object_2D::ComputeMeanAndStandardFrame, Object.cc:63-102
  static void frame_mean(Obj2D* f) {
    for (auto it = f->pts.begin(); it != f->pts.end();) {
      if ((*it)->bad) {
        for (int a = 0; a < 3; a++) f->sum[a] -= (*it)->pos[a];
        it = f->pts.erase(it);
      } else
        ++it;
    }
    const float sc = (float)(1. / (double)f->pts.size());
    for (int a = 0; a < 3; a++) f->pos[a] = f->sum[a] * sc + 0.0f;
    float s2[3] = {0, 0, 0};
    for (auto* p : f->pts) {
      if (p->bad) continue;
      for (int a = 0; a < 3; a++) s2[a] += (p->pos[a] - f->pos[a]) * (p->pos[a] - f->pos[a]);
    }
    for (int a = 0; a < 3; a++) f->std_[a] = std::sqrt(s2[a] / (float)f->pts.size());
  }

  // Object_2D::RemoveOutliersByBoxPlot, Object.cc:106-158
  void boxplot(Obj2D* f) {
    std::vector<float> zc;
    for (auto* p : f->pts) {
      float pc[3];
      transform_point(T, p->pos, pc);
      zc.push_back(pc[2]);
    }
    std::sort(zc.begin(), zc.end());
    if ((zc.size() / 4 <= 0) || (zc.size() * 3 / 4 >= zc.size() - 1)) return;
    float Q1 = zc[zc.size() / 4];
    float Q3 = zc[zc.size() * 3 / 4];
    float IQR = Q3 - Q1;
    float max_th = (float)(Q3 + 1.5 * IQR);
    for (auto it = f->pts.begin(); it != f->pts.end();) {
      float pc[3];
      transform_point(T, (*it)->pos, pc);
      if (pc[2] > max_th) it = f->pts.erase(it);
      else ++it;
    }
    frame_mean(f);
  }

  bool overlap(ObjMap* a, ObjMap* b) {  // Object_Map::WhetherOverlap, :1906-1922
    float dx = (float)std::fabs(a->cub.center[0] - b->cub.center[0]);
    float dy = (float)std::fabs(a->cub.center[1] - b->cub.center[1]);
    float dz = (float)std::fabs(a->cub.center[2] - b->cub.center[2]);
    float sl = a->cub.lenth / 2 + b->cub.lenth / 2;
    float sw = a->cub.width / 2 + b->cub.width / 2;
    float sh = a->cub.height / 2 + b->cub.height / 2;
    return (dx < sl) && (dy < sw) && (dz < sh);
  }

  struct NPLog {
    int det, obj;
    NPResult r;
  };
  struct TLog {
    int det, obj;
    float tx, ty, tz;
  };
  std::vector<NPLog> np_log;
  std::vector<TLog> t_log;

  // TrackWithMotionModel object section, Tracking.cc:1241-1696
  void frame(unsigned long fid, const float* Tcw, int nb, const int32_t* boxes, int npts,
             const int32_t* ids, const float* pos, const float* uv, const uint8_t* bad, int32_t* out) {
    cur_id = fid;
    std::memcpy(T, Tcw, sizeof(T));
    np_log.clear();
    t_log.clear();
    std::vector<Obj2D*> o2;
    for (int k = 0; k < nb; k++) {
      Obj2D* f = new Obj2D();
      all2d.push_back(f);
      f->class_id = boxes[5 * k];
      f->bx = boxes[5 * k + 1];
      f->by = boxes[5 * k + 2];
      f->bw = boxes[5 * k + 3];
      f->bh = boxes[5 * k + 4];
      f->box = Rect(f->bx, f->by, f->bw, f->bh);
      f->input_index = k;
      f->method = 0;
      o2.push_back(f);
      out[4 * k] = -1;
      out[4 * k + 1] = -1;
      out[4 * k + 2] = f->class_id;
      out[4 * k + 3] = 0;
    }
    // map points of this frame (create or refresh)
    std::vector<MapPoint*> tracked(npts);
    for (int i = 0; i < npts; i++) {
      auto it = mps.find(ids[i]);
      MapPoint* p;
      if (it == mps.end()) {
        p = new MapPoint();
        p->id = ids[i];
        mps[ids[i]] = p;
      } else
        p = it->second;
      for (int a = 0; a < 3; a++) p->pos[a] = pos[3 * i + a];
      p->bad = bad ? bad[i] != 0 : false;
      tracked[i] = p;
    }
    // STEP 2 AssociateObjAndPoints, Tracking.cc:2434-2468
    for (int i = 0; i < npts; i++) {
      MapPoint* p = tracked[i];
      if (p->bad) continue;
      for (auto* f : o2) {
        if (f->box.contains(uv[2 * i], uv[2 * i + 1])) {
          p->feat_u = uv[2 * i];
          p->feat_v = uv[2 * i + 1];
          f->pts.push_back(p);
          for (int a = 0; a < 3; a++) f->sum[a] += p->pos[a];
        }
      }
    }
    // STEP 3 AssociateObjAndLines (Tracking.cc:1286): the frame's staged line set
    {
      static const std::vector<float> none;
      const std::vector<float>& fl = staged_next < staged_lines.size() ? staged_lines[staged_next] : none;
      associate_lines(o2, fl);
      if (staged_next < staged_lines.size() && ++staged_next == staged_lines.size()) {
        staged_lines.clear();
        staged_next = 0;
      }
    }
    // STEP 4
    for (auto* f : o2) {
      frame_mean(f);
      if (f->pts.size() < 8) continue;
      boxplot(f);
    }
    // STEP 5
    for (auto* f : o2) {
      const float sc = (float)(1. / (double)f->pts.size());
      for (int a = 0; a < 3; a++) f->pos[a] = f->sum[a] * sc + 0.0f;
      std::vector<float> xs, ys;
      for (auto* p : f->pts) {
        xs.push_back(p->feat_u);
        ys.push_back(p->feat_v);
      }
      if (xs.size() < 4) continue;
      std::sort(xs.begin(), xs.end());
      std::sort(ys.begin(), ys.end());
      float x_min = xs[0], x_max = xs.back(), y_min = ys[0], y_max = ys.back();
      if (x_min < 0) x_min = 0;
      if (y_min < 0) y_min = 0;
      if (x_max > cam.cols) x_max = (float)cam.cols;
      if (y_max > cam.rows) y_max = (float)cam.rows;
      f->feat_rect = rect_from_floats(x_min, y_min, x_max - x_min, y_max - y_min);
    }
    // STEP 6 filters, Tracking.cc:1383-1487
    for (size_t a = 0; a < o2.size(); a++) {
      int num = 0;
      for (size_t b = 0; b < o2.size(); b++) {
        if (a == b) continue;
        if (latter(o2[a]->box, o2[b]->box) > 0.05) num++;
      }
      if (num > 4) o2[a]->bad = true;
    }
    for (size_t a = 0; a < o2.size(); a++) {
      Obj2D* f = o2[a];
      if (f->bad) continue;
      if (f->class_id == 0 || f->class_id == 63 || f->class_id == 15) f->bad = true;
      if ((float)f->box.area() / (float)(cam.cols * cam.rows) > 0.5) f->bad = true;
      if (f->pts.size() < 5)
        f->bad = true;
      else if (f->pts.size() >= 5 && f->pts.size() < 10) {
        if (f->bx < 20 || f->by < 20 || f->bx + f->bw > cam.cols - 20 || f->by + f->bh > cam.rows - 20)
          f->bad = true;
      }
      if (f->bx < 5 || f->by < 5 || f->bx + f->bw > cam.cols - 5 || f->by + f->bh > cam.rows - 5)
        f->on_edge = true;
      for (size_t b = 0; b < o2.size(); b++) {
        if (o2[b]->bad) continue;
        if (a == b) continue;
        if (iou(f->box, o2[b]->box) > 0.3) {
          if (f->score < o2[b]->score) f->bad = true;
          else if (f->score >= o2[b]->score) o2[b]->bad = true;
        }
        if (iou(f->box, o2[b]->box) > 0.05) {
          if (former(f->box, o2[b]->box) > 0.85) f->bad = true;
          if (latter(f->box, o2[b]->box) > 0.85) o2[b]->bad = true;
        }
      }
    }
    std::vector<Obj2D*> kept;
    for (auto* f : o2) {
      if (!f->bad) kept.push_back(f);
      else f->method = -1;
    }
    // STEP 7/8: dead in the reference (Q10)
    // STEP 9 InitObjMap, Tracking.cc:2531-2598
    if (!ini) {
      int good = -1;
      for (auto* f : kept) {
        if (f->pts.size() < 10) {
          f->few = true;
          f->current = false;
          f->method = 6;
          continue;
        }
        good++;
        ini = true;
        ini_frame = (long)fid;
        ObjMap* o = new ObjMap();
        o->frames.push_back(f);
        o->mnId = good;
        o->mnClass = f->class_id;
        o->confidence = 1;
        o->first_observe = true;
        o->added = o->last_add = o->lastlast_add = (int)fid;
        o->last = f->box;
        for (int a = 0; a < 3; a++) {
          o->sum[a] = f->sum[a];
          o->center[a] = f->pos[a];
        }
        for (auto* p : f->pts) {
          p->object_id = o->mnId;
          p->object_class = o->mnClass;
          p->object_id_vector.insert(std::make_pair(o->mnId, 1));
          o->pts.push_back(p);
        }
        f->mnId = o->mnId;
        f->which_time = o->confidence;
        f->current = true;
        f->method = 7;
        f->alias = o;
        mean_and_standard(o);
        objs.push_back(o);
      }
    }
    // STEP 10
    if ((long)fid > ini_frame && ini) {
      for (auto* o : objs) {
        if (o->bad) continue;
        if ((unsigned long)(long)o->last_add > fid - 30)
          project_rect(o);
        else
          o->proj = Rect(0, 0, 0, 0);
      }
      for (auto* f : kept) {
        if (f->pts.size() < 5) {
          f->few = true;
          f->current = false;
          f->method = 6;
          continue;
        }
        associate(f);
      }
      for (int i = (int)objs.size() - 1; i >= 0; i--) {
        if (flag == "NA") continue;
        ObjMap* o = objs[i];
        if (o->bad) continue;
        int df = (int)o->frames.size();
        if (df < 10) {
          if ((unsigned long)(long)o->last_add < (fid - 30)) {
            if (df < 5)
              o->bad = true;
            else {
              bool ov = false;
              for (int j = (int)objs.size() - 1; j >= 0; j--) {
                if (objs[j]->bad || i == j) continue;
                if (overlap(o, objs[j])) {
                  ov = true;
                  break;
                }
              }
              if (ov) o->bad = true;
            }
          }
        }
      }
      for (int i = (int)objs.size() - 1; i >= 0; i--) {
        if ((unsigned long)(long)objs[i]->last_add != fid) continue;
        for (int j = (int)objs.size() - 1; j >= 0; j--) {
          if (i == j) continue;
          if ((unsigned long)(long)objs[j]->last_add == fid) {
            auto& m = objs[i]->sametime;
            auto it = m.find(objs[j]->mnId);
            if (it != m.end()) it->second += 1;
            else m[objs[j]->mnId] = 1;
          }
        }
      }
      // step 10.6 SampleObjYaw for regular objects seen this frame (Tracking.cc:1650-1671)
      for (int i = (int)objs.size() - 1; i >= 0; i--) {
        ObjMap* o = objs[i];
        if (o->bad) continue;
        if ((unsigned long)(long)o->last_add < fid - 5) continue;
        const int c = o->mnClass;
        if (c == 73 || c == 64 || c == 65 || c == 66 || c == 56)
          if ((unsigned long)(long)o->last_add == fid) sample_yaw(o);
      }
    }
    for (auto* f : o2) {
      int k = f->input_index;
      out[4 * k] = f->method;
      out[4 * k + 1] = f->mnId;
      out[4 * k + 3] = (int)f->pts.size();
    }
  }

  // ---- LocalMapping object maintenance, LocalMapping.cc:772-882
  bool double_ttest(ObjMap* a, ObjMap* b) {  // Object.cc:1659-1712 (Q5)
    int n1 = (int)a->frames.size(), n2 = (int)b->frames.size();
    float d[3], t[3];
    for (int k = 0; k < 3; k++) {
      float m1 = a->center[k], m2 = b->center[k];
      d[k] = std::sqrt(((((float)(n1 - 1) * m1 * m1) + ((float)(n2 - 1) * m2 * m2)) / (float)(n1 + n2 - 2)) *
                       (float)(1 / n1 + 1 / n2));
      t[k] = (m1 - m2) / d[k];
    }
    const float* row = kTTable[std::min(n1 + n2 - 2, 121)];
    return t[0] < row[5] && t[1] < row[5] && t[2] < row[5];
  }

  void merge(ObjMap* a, ObjMap* b) {  // Object_Map::MergeTwoMapObjs, :1716-1902
    for (auto* p : b->pts) {
      double v[3] = {p->pos[0], p->pos[1], p->pos[2]}, s[3];
      pose_inverse_apply(a->cub.q, a->cub.t, v, s);
      if (std::fabs(s[0]) > 1.1 * a->cub.lenth / 2 || std::fabs(s[1]) > 1.1 * a->cub.width / 2 ||
          std::fabs(s[2]) > 1.1 * a->cub.height / 2)
        continue;
      p->object_id = a->mnId;
      p->object_class = a->mnClass;
      vote(p, p->object_id);
      bool new_point = true;
      for (auto* q : a->pts)
        if (same_pos(p, q)) {
          new_point = false;
          break;
        }
      if (new_point) {
        a->pts.push_back(p);
        for (int k = 0; k < 3; k++) a->sum[k] += p->pos[k];
      }
    }
    for (auto* f : b->frames) {
      f->mnId = a->mnId;
      a->confidence++;
      a->frames.push_back(f);
    }
    for (auto& kv : b->sametime) {
      auto it = a->sametime.find(kv.first);
      if (it != a->sametime.end()) it->second = it->second + kv.second;
      else a->sametime[kv.first] = 1;
    }
    int oLast = a->last_add, oLastLast = a->lastlast_add;
    Rect oRect = a->last;
    if (a->last_add > b->last_add) {
      if (oLastLast > b->last_add) {
      } else {
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
        // Q29: reference indexes size()-2, UB for a one-frame object; use front().
        a->lastlast = b->frames.size() >= 2 ? b->frames[b->frames.size() - 2]->box : b->frames.front()->box;
      }
    }
    // step 5. orientation measurements (Object.cc:1842-1901)
    const int c = a->mnClass;
    if (c == 73 || c == 64 || c == 65 || c == 66 || c == 56) {
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
        for (int i = 0; i < std::min(6, (int)a->angles.size()); i++) {
          const float f = a->angles[i][2];
          if (f > best_score) {
            best_score = f;
            best = i;
          }
        }
        a->cub.rotY = a->angles[best][0];
        a->cub.err_parallel = a->angles[best][3];
        a->cub.err_yaw = a->angles[best][4];
        update_pose(a);
      }
    }
  }

  void whether_merge(ObjMap* o) {  // Object_Map::WhetherMergeTwoMapObjs, :1607-1655
    for (auto& kv : o->reobj) {
      int nObjId = kv.first;
      if (kv.second < 3) continue;
      if (objs[nObjId]->bad) continue;
      bool dt = double_ttest(o, objs[nObjId]);
      bool same = true;
      if (o->sametime.find(nObjId) != o->sametime.end())
        continue;
      else
        same = false;
      if (!same || dt) {
        int n1 = (int)o->frames.size(), n2 = (int)objs[nObjId]->frames.size();
        if (n1 > n2) {
          merge(o, objs[nObjId]);
          mean_and_standard(o);
          iforest_delete(o);
          objs[nObjId]->bad = true;
        } else {
          merge(objs[nObjId], o);
          mean_and_standard(objs[nObjId]);
          iforest_delete(objs[nObjId]);
          o->bad = true;
        }
      }
    }
  }

  void divide_equally(ObjMap* a, ObjMap* b, float ox, float oy, float oz) {  // :2044-2073
    for (auto it = a->pts.begin(); it != a->pts.end();) {
      const float* P = (*it)->pos;
      const Cuboid& c = b->cub;
      if ((P[0] > c.center[0] - (c.lenth / 2 - ox / 2) && P[0] < c.center[0] + (c.lenth / 2 - ox / 2)) &&
          (P[1] > c.center[1] - (c.width / 2 - oy / 2) && P[1] < c.center[1] + (c.width / 2 - oy / 2)) &&
          (P[2] > c.center[2] - (c.height / 2 - oz / 2) && P[2] < c.center[2] + (c.height / 2 - oz / 2)))
        it = a->pts.erase(it);
      else
        ++it;
    }
  }

  void big_to_small(ObjMap* a, ObjMap* s) {  // :1926-2040 (the direction flags are dead)
    for (auto it = a->pts.begin(); it != a->pts.end();) {
      const float* P = (*it)->pos;
      const Cuboid& c = s->cub;
      if (P[0] > c.x_min && P[0] < c.x_max && P[1] > c.y_min && P[1] < c.y_max && P[2] > c.z_min &&
          P[2] < c.z_max)
        it = a->pts.erase(it);
      else
        ++it;
    }
    mean_and_standard(a);
  }

  void deal_overlap(ObjMap* a, ObjMap* b, float ox, float oy, float oz) {  // :2077-2178
    float va = (a->cub.lenth * a->cub.width) * a->cub.height;
    float vb = (b->cub.lenth * b->cub.width) * b->cub.height;
    float ov = (ox * oy) * oz;
    bool bIou = (ov / (va + vb - ov)) >= 0.3;
    bool bVolume = (va > 2 * vb) || (vb > 2 * va);
    bool bSame = false;
    auto it = a->sametime.find(b->mnId);
    if (it != a->sametime.end()) bSame = it->second > 3;
    bool bClass = a->mnClass == b->mnClass;
    if (bIou && !bVolume && !bSame && bClass) {
      if (a->frames.size() >= b->frames.size()) {
        merge(a, b);
        b->bad = true;
      } else {
        merge(b, a);
        a->bad = true;
      }
    } else if (bVolume && !bSame && bClass) {
      if (a->frames.size() >= b->frames.size() && va > vb)
        b->bad = true;
      else if (a->frames.size() < b->frames.size() && va < vb)
        a->bad = true;
    } else if (bIou && !bVolume && bSame && bClass) {
      divide_equally(a, b, ox, oy, oz);
      divide_equally(b, b, ox, oy, oz);
      mean_and_standard(a);
      mean_and_standard(b);
    } else if (!bIou && bVolume && bSame && !bClass) {
      if (va > vb) big_to_small(a, b);
      else if (va < vb) big_to_small(b, a);
    } else if (bIou && !bSame && bClass) {
      if (a->frames.size() / 2 >= b->frames.size()) {
        merge(a, b);
        b->bad = true;
      } else if (b->frames.size() / 2 >= a->frames.size()) {
        merge(b, a);
        a->bad = true;
      }
    }
  }

  void local_mapping() {
    // UpdateObject, LocalMapping.cc:772-795
    for (auto* o : objs) {
      if (o->pts.size() < 10 || o->bad) continue;
      mean_and_standard(o);
    }
    if (flag == "NA" || flag == "IoU" || flag == "NP") return;
    // MergePotentialAssObjs, :799-824
    for (auto* o : objs) {
      if (o->bad) continue;
      if (o->frames.size() >= 10 && o->reobj.size() > 0) whether_merge(o);
    }
    // WhetherOverlapObject, :828-882
    for (size_t i = 0; i < objs.size(); i++) {
      ObjMap* a = objs[i];
      if (a->pts.size() < 10 || a->bad || a->frames.size() < 10) continue;
      for (size_t j = 0; j < objs.size(); j++) {
        if (i == j) continue;
        ObjMap* b = objs[j];
        if (b->pts.size() < 10 || b->bad || b->frames.size() < 10) continue;
        float dx = (float)std::fabs(a->cub.center[0] - b->cub.center[0]);
        float dy = (float)std::fabs(a->cub.center[1] - b->cub.center[1]);
        float dz = (float)std::fabs(a->cub.center[2] - b->cub.center[2]);
        float sl = a->cub.lenth / 2 + b->cub.lenth / 2;
        float sw = a->cub.width / 2 + b->cub.width / 2;
        float sh = a->cub.height / 2 + b->cub.height / 2;
        if (dx < sl && dy < sw && dz < sh) deal_overlap(a, b, sl - dx, sw - dy, sh - dz);
      }
    }
  }
};

}  // namespace orc

using namespace orc;

struct orc_replay {
  Replay r;
};

extern "C" {

int orc_np_test(int m_total, const float* frame_pts, const uint8_t* frame_valid, int n_total,
                const float* obj_pts, const uint8_t* obj_valid, orc_np_stats* out) {
  std::vector<const float*> fv, ov;
  for (int i = 0; i < m_total; i++)
    if (!frame_valid || frame_valid[i]) fv.push_back(frame_pts + 3 * i);
  for (int i = 0; i < n_total; i++)
    if (!obj_valid || obj_valid[i]) ov.push_back(obj_pts + 3 * i);
  NPResult R = np_test(fv, n_total, ov);
  out->verdict = R.verdict;
  out->m = R.m;
  out->n = R.n;
  for (int a = 0; a < 3; a++) {
    out->w[a] = R.w[a];
    out->cnt_gt[a] = R.gt[a];
    out->cnt_lt[a] = R.lt[a];
    out->cnt_eq[a] = R.eq[a];
  }
  out->r1 = R.r1;
  out->r2 = R.r2;
  return R.verdict;
}

int orc_iforest_scores(const float* pts, int n, uint32_t trees, uint32_t seed, uint32_t sample_size,
                       double* scores) {
  std::vector<double> s;
  if (!iforest_scores(pts, (uint32_t)n, trees, seed, sample_size, s)) return -1;
  std::copy(s.begin(), s.end(), scores);
  return 0;
}

void orc_mt19937_stream(uint32_t seed, int n, uint32_t* out) {
  MT19937 g(seed);
  for (int i = 0; i < n; i++) out[i] = g();
}
uint32_t orc_lemire_u32(uint32_t seed, int n_draws, uint32_t range, uint32_t* out) {
  MT19937 g(seed);
  for (int i = 0; i < n_draws; i++) out[i] = lemire(g, range);
  return 0;
}
int orc_shuffle_ids(uint32_t seed, int n, uint32_t* ids) {
  MT19937 g(seed);
  std::vector<uint32_t> v(n);
  for (int i = 0; i < n; i++) v[i] = (uint32_t)i;
  shuffle_ids(v, g);
  std::copy(v.begin(), v.end(), ids);
  return 0;
}
void orc_canonical_float(uint32_t seed, int n, float lo, float hi, float* out) {
  MT19937 g(seed);
  for (int i = 0; i < n; i++) out[i] = uniform_real(g, lo, hi);
}

float orc_bbox_iou(const int* a, const int* b) {
  return iou(Rect(a[0], a[1], a[2], a[3]), Rect(b[0], b[1], b[2], b[3]));
}
float orc_bbox_former(const int* a, const int* b) {
  return former(Rect(a[0], a[1], a[2], a[3]), Rect(b[0], b[1], b[2], b[3]));
}
float orc_bbox_latter(const int* a, const int* b) {
  return latter(Rect(a[0], a[1], a[2], a[3]), Rect(b[0], b[1], b[2], b[3]));
}

int orc_project_rect(const orc_camera* cam, const float* Tcw, int n, const float* pts, int* rect) {
  if (n <= 0) return -1;
  Cam c{cam->fx, cam->fy, cam->cx, cam->cy, cam->img_w, cam->img_h};
  std::vector<float> xs, ys;
  for (int i = 0; i < n; i++) {
    float u, v;
    project(c, Tcw, pts + 3 * i, u, v);
    xs.push_back(u);
    ys.push_back(v);
  }
  std::sort(xs.begin(), xs.end());
  std::sort(ys.begin(), ys.end());
  float x_min = xs[0], x_max = xs.back(), y_min = ys[0], y_max = ys.back();
  if (x_min < 0) x_min = 0;
  if (y_min < 0) y_min = 0;
  if (x_max > c.cols) x_max = (float)c.cols;
  if (y_max > c.rows) y_max = (float)c.rows;
  Rect r = rect_from_floats(x_min, y_min, x_max - x_min, y_max - y_min);
  rect[0] = r.x;
  rect[1] = r.y;
  rect[2] = r.w;
  rect[3] = r.h;
  return 0;
}

orc_replay* orc_replay_create(const char* flag, int img_w, int img_h, const float* K4) {
  orc_replay* r = new orc_replay();
  r->r.flag = flag;
  r->r.cam = Cam{K4[0], K4[1], K4[2], K4[3], img_w, img_h};
  return r;
}
void orc_replay_destroy(orc_replay* r) { delete r; }

int orc_replay_frame(orc_replay* r, int frame_id, const float* Tcw, int n_boxes, const int32_t* boxes,
                     int n_pts, const int32_t* mp_ids, const float* mp_pos, const float* kp_uv,
                     const uint8_t* mp_bad, int32_t* det_out) {
  r->r.frame((unsigned long)frame_id, Tcw, n_boxes, boxes, n_pts, mp_ids, mp_pos, kp_uv, mp_bad, det_out);
  return (int)r->r.objs.size();
}
int orc_replay_lines(orc_replay* r, int n_frames, const int32_t* n_lines, const float* lines) {
  for (int t = 0; t < n_frames; t++) {
    r->r.staged_lines.emplace_back(lines, lines + 4 * (size_t)n_lines[t]);
    lines += 4 * (size_t)n_lines[t];
  }
  return 0;
}
int orc_replay_local_mapping(orc_replay* r) {
  r->r.local_mapping();
  return 0;
}
// LocalMapping's map-point changes (LocalBundleAdjustment SetWorldPos, MapPointCulling /
// KeyFrameCulling SetBadFlag, SearchInNeighbors Replace -- LocalMapping.cc:60-80,
// MapPoint.cc:73-77,151-220) for points the replay knows. The object code reads them
// live: GetWorldPos() / isBad() at every later ComputeMeanAndStandard (Object.cc:967-992),
// NP test, projected rect, forest and duplicate check. Replace(pMP) leaves the object
// holding the old, now bad, pointer (no membership transfer), so it is a bad flag here.
int orc_replay_update_points(orc_replay* r, int n, const int32_t* ids, const float* pos, const uint8_t* bad) {
  for (int i = 0; i < n; i++) {
    auto it = r->r.mps.find(ids[i]);
    if (it == r->r.mps.end()) continue;  // never tracked: no object or detection holds it
    MapPoint* p = it->second;
    if (pos)
      for (int a = 0; a < 3; a++) p->pos[a] = pos[3 * i + a];
    if (bad) p->bad = bad[i] != 0;
  }
  return 0;
}
int orc_replay_num_objects(orc_replay* r) { return (int)r->r.objs.size(); }
int orc_replay_object(orc_replay* r, int i, int32_t* ints, float* floats) {
  if (i < 0 || i >= (int)r->r.objs.size()) return -1;
  ObjMap* o = r->r.objs[i];
  ints[0] = o->mnId;
  ints[1] = o->mnClass;
  ints[2] = o->bad;
  ints[3] = (int)o->frames.size();
  ints[4] = (int)o->pts.size();
  ints[5] = o->last_add;
  ints[6] = (int)o->reobj.size();
  ints[7] = (int)o->sametime.size();
  for (int a = 0; a < 3; a++) {
    floats[a] = o->center[a];
    floats[3 + a] = o->std_[a];
    floats[6 + a] = o->cstd[a];
  }
  floats[9] = o->cub.lenth;
  floats[10] = o->cub.width;
  floats[11] = o->cub.height;
  floats[12] = o->cub.rmax;
  floats[13] = o->cstd_all;
  floats[14] = (float)o->proj.x;
  floats[15] = (float)o->proj.w;
  floats[16] = o->cub.rotY;
  floats[17] = (float)o->angles.size();
  floats[18] = o->cub.err_parallel;
  floats[19] = o->cub.err_yaw;
  return 0;
}
int orc_replay_object_points(orc_replay* r, int i, int32_t* ids, int cap) {
  if (i < 0 || i >= (int)r->r.objs.size()) return -1;
  ObjMap* o = r->r.objs[i];
  int n = (int)o->pts.size();
  for (int k = 0; k < n && k < cap; k++) ids[k] = o->pts[k]->id;
  return n;
}

}  // extern "C"
