// lines_ref.cpp -- CPU restatement of the per-frame line detection of the EAO Frame
// (TEST INFRASTRUCTURE ONLY: the checker of tests/, never linked by the product).
//
//   Frame.cc:324-328       line_lbd_detect::detect_raw_lines(rawImage, keylines_raw)  (use_LSD = false)
//                          line_lbd_detect::filter_lines(keylines_raw, keylines_out)  (octave 0, length > 50)
//                          keylines_to_mat(keylines_out, all_lines_mat, 1)
//   line_lbd_allclass.cpp:137-214, BinaryDescriptor::detectImpl / OctaveKeyLines
//   (src/line_detect/libs/binary_descriptor.cpp:486-589, 796-1148) with numOfOctave_ = 1
//   (Tracking.cc:161-163): GaussianBlur(5x5, sigma 1) then EDLineDetector::EDline
//   (binary_descriptor.cpp:1583-2630: EdgeDrawing, LeastSquaresLineFit_, LineValidation_),
//   nfa / log_gamma (include/line_lbd/line_descriptor/descriptor.hpp:649-844).
//
// OpenCV 3.2 primitive semantics restated (OpenCV is absent here, so
// the parity of this restatement against the original binary is UNPINNED):
//   GaussianBlur 8U -> the fixed-point separable path (taps cvRound(k * 256), rows in int,
//   columns (s + 2^15) >> 16, saturated), BORDER_REFLECT_101 on the isolated image;
//   Sobel(CV_16S, ksize 3) -> [-1 0 1] x [1 2 1], exact in integers, REFLECT_101;
//   threshold(TOZERO, 81) on 16S; Mat / 4 -> saturate_cast<short>(v * 0.25f) (cvRound,
//   half to even); compare(CMP_LT) -> 255 / 0.
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "oracle.h"

namespace {

constexpr int kHorizontal = 255, kVertical = 0;  // binary_descriptor.cpp:58-59
constexpr int kUp = 1, kRight = 2, kDown = 3, kLeft = 4;
// EDLineDetector's knobs; the defaults are EDLineDetector() (:1518-1524), the detector the EAO
// Frame runs. Other values serve only the pinning of this restatement against the Edge Drawing
// library's own outputs (tests/test_oracle_ed_pin.py).
struct EdParams {
  int grad_th = 80, anchor_th = 8, scan = 2, min_line_len = 15;
  double fit_err_th = 1.6;
  int gdiv = 4;  // gImg_ = thresholded |dx| + |dy| divided by this (EdgeDrawing, :1650-1662)
  int validate = 1;  // 0: keep every fitted segment (bValidate_ = false, :2590-2600)
};
const EdParams kDefaultParams{};
constexpr int kTryTime = 6, kSkip = 2;  // :64-65

inline int reflect101(int p, int len) {
  if (len == 1) return 0;
  while (p < 0 || p >= len) {
    if (p < 0) p = -p;
    if (p >= len) p = 2 * len - 2 - p;
  }
  return p;
}
inline int round_half_even(double v) { return (int)std::nearbyint(v); }

// getGaussianKernel(5, 1, CV_32F) -> the integer taps of the 8U separable path
void gauss_kernel5(int* k) {
  float cf[5];
  double sum = 0;
  const double sigma = 1.0, scale2X = -0.5 / (sigma * sigma);
  for (int i = 0; i < 5; i++) {
    const double x = i - (5 - 1) * 0.5;
    cf[i] = (float)std::exp(scale2X * x * x);
    sum += cf[i];
  }
  sum = 1. / sum;
  for (int i = 0; i < 5; i++) {
    cf[i] = (float)(cf[i] * sum);
    k[i] = round_half_even((double)cf[i] * 256.0);
  }
}

double log_gamma_lanczos(double x) {  // descriptor.hpp:694-707
  static const double q[7] = {75122.6331530, 80916.6278952, 36308.2951477, 8687.24529705,
                              1168.92649479, 83.8676043424, 2.50662827511};
  double a = (x + 0.5) * std::log(x + 5.5) - (x + 5.5);
  double b = 0.0;
  for (int n = 0; n < 7; n++) {
    a -= std::log(x + (double)n);
    b += q[n] * std::pow(x, (double)n);
  }
  return a + std::log(b);
}
double log_gamma_windschitl(double x) {  // :724-727
  return 0.918938533204673 + (x - 0.5) * std::log(x) - x +
         0.5 * x * std::log(x * std::sinh(1 / x) + 1 / (810.0 * std::pow(x, 6.0)));
}
double log_gamma(double x) { return x > 15.0 ? log_gamma_windschitl(x) : log_gamma_lanczos(x); }
bool double_equal(double a, double b) {  // :649-670
  if (a == b) return true;
  const double abs_diff = std::fabs(a - b), aa = std::fabs(a), bb = std::fabs(b);
  double abs_max = aa > bb ? aa : bb;
  if (abs_max < DBL_MIN) abs_max = DBL_MIN;
  return (abs_diff / abs_max) <= (100.0 * DBL_EPSILON);
}
double nfa(int n, int k, double p, double logNT) {  // :763-844
  const double tolerance = 0.1;
  if (n == 0 || k == 0) return -logNT;
  if (n == k) return -logNT - (double)n * std::log10(p);
  const double p_term = p / (1.0 - p);
  const double log1term = log_gamma((double)n + 1.0) - log_gamma((double)k + 1.0) -
                          log_gamma((double)(n - k) + 1.0) + (double)k * std::log(p) +
                          (double)(n - k) * std::log(1.0 - p);
  double term = std::exp(log1term);
  if (double_equal(term, 0.0)) {
    if ((double)k > (double)n * p) return -log1term / 2.30258509299404568402 - logNT;
    return -logNT;
  }
  double bin_tail = term;
  for (int i = k + 1; i <= n; i++) {
    const double bin_term = (double)(n - i + 1) / (double)i;
    const double mult_term = bin_term * p_term;
    term *= mult_term;
    bin_tail += term;
    if (bin_term < 1.0) {
      const double err = term * ((1.0 - std::pow(mult_term, (double)(n - i + 1))) / (1.0 - mult_term) - 1.0);
      if (err < tolerance * std::fabs(-std::log10(bin_tail) - logNT) * bin_tail) break;
    }
  }
  return -std::log10(bin_tail) - logNT;
}

struct Maps {
  int w = 0, h = 0;
  std::vector<uint8_t> blur;
  std::vector<int16_t> dx, dy, g;  // g: thresholded gradient / 4 (gImg_)
  std::vector<uint8_t> dir;        // dirImg_: 255 = Horizontal
};

void compute_maps(const uint8_t* gray, int w, int h, Maps& M, const EdParams& P = kDefaultParams) {
  M.w = w;
  M.h = h;
  const size_t n = (size_t)w * h;
  M.blur.assign(n, 0);
  M.dx.assign(n, 0);
  M.dy.assign(n, 0);
  M.g.assign(n, 0);
  M.dir.assign(n, 0);
  int k[5];
  gauss_kernel5(k);
  std::vector<int> R(n);
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      int s = 0;
      for (int i = 0; i < 5; i++) s += k[i] * gray[(size_t)y * w + reflect101(x + i - 2, w)];
      R[(size_t)y * w + x] = s;
    }
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      int s = 0;
      for (int j = 0; j < 5; j++) s += k[j] * R[(size_t)reflect101(y + j - 2, h) * w + x];
      int v = (s + (1 << 15)) >> 16;
      M.blur[(size_t)y * w + x] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
    }
  const uint8_t* B = M.blur.data();
  auto px = [&](int x, int y) { return (int)B[(size_t)reflect101(y, h) * w + reflect101(x, w)]; };
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      const int gx = (px(x + 1, y - 1) - px(x - 1, y - 1)) + 2 * (px(x + 1, y) - px(x - 1, y)) +
                     (px(x + 1, y + 1) - px(x - 1, y + 1));
      const int gy = (px(x - 1, y + 1) - px(x - 1, y - 1)) + 2 * (px(x, y + 1) - px(x, y - 1)) +
                     (px(x + 1, y + 1) - px(x + 1, y - 1));
      const size_t i = (size_t)y * w + x;
      M.dx[i] = (int16_t)gx;
      M.dy[i] = (int16_t)gy;
      const int ax = gx < 0 ? -gx : gx, ay = gy < 0 ? -gy : gy, s = ax + ay;
      const int t = s > P.grad_th + 1 ? s : 0;
      M.g[i] = P.gdiv == 4 ? (int16_t)round_half_even((double)((float)t * 0.25f))
                           : (int16_t)std::min(t / P.gdiv, 32767);
      M.dir[i] = ax < ay ? kHorizontal : kVertical;
    }
}

struct Chains {
  std::vector<uint32_t> x, y, sid;  // sid: numOfEdges + 1 offsets
};

// EdgeDrawing, binary_descriptor.cpp:1583-2381
int edge_drawing(const Maps& M, Chains& E, std::vector<uint32_t>* anchors_out,
                 const EdParams& P = kDefaultParams) {
  const int W = M.w, H = M.h;
  const uint32_t pixelNum = (uint32_t)W * H;
  const uint32_t edgePixelArraySize = pixelNum / 5, maxNumOfEdge = edgePixelArraySize / 20;
  const int16_t* pg = M.g.data();
  const uint8_t* pd = M.dir.data();
  std::vector<uint32_t> ax, ay;
  for (int w = 1; w < W - 1; w += P.scan)
    for (int h = 1; h < H - 1; h += P.scan) {
      const int i = h * W + w;
      if (pd[i] == kHorizontal) {
        if (pg[i] >= pg[i - W] + P.anchor_th && pg[i] >= pg[i + W] + P.anchor_th) {
          ax.push_back(w);
          ay.push_back(h);
        }
      } else if (pg[i] >= pg[i - 1] + P.anchor_th && pg[i] >= pg[i + 1] + P.anchor_th) {
        ax.push_back(w);
        ay.push_back(h);
      }
    }
  if (anchors_out) {
    anchors_out->clear();
    for (size_t i = 0; i < ax.size(); i++) anchors_out->push_back(ay[i] * W + ax[i]);
  }
  if (ax.size() > edgePixelArraySize) return -1;
  std::vector<uint8_t> edge(pixelNum, 0);
  std::vector<uint32_t> fX(edgePixelArraySize + 1), fY(edgePixelArraySize + 1), sX(edgePixelArraySize + 1),
      sY(edgePixelArraySize + 1), fS(maxNumOfEdge + 2), sS(maxNumOfEdge + 2);
  uint32_t offF = 0, offS = 0, offPS = 0;
  uint32_t lastX = 0, lastY = 0;  // persist across walks and anchors, as in the reference
  // one walk from (x, y) with initial direction dir0, pixels appended to (X, Y, off)
  // the walk reads gImg_ as unsigned char (gValue1..3, :1643, 1746-2000): /4 values above 255
  // wrap; the unscaled (gdiv 1) pinning variant compares the full values, as ED does
  auto gv = [&](int i) { return P.gdiv == 4 ? (int)(uint8_t)pg[i] : (int)pg[i]; };
  auto walk = [&](uint32_t x, uint32_t y, int lastDir, std::vector<uint32_t>& X, std::vector<uint32_t>& Y,
                  uint32_t& off) -> bool {
    int idx = (int)(y * W + x);
    while (pg[idx] > 0 && !edge[idx]) {
      if (off >= edgePixelArraySize) return false;  // the reference overruns its array here
      edge[idx] = 1;
      X[off] = x;
      Y[off++] = y;
      int should = 0;
      if (pd[idx] == kHorizontal) {
        if (lastDir == kUp || lastDir == kDown) should = x > lastX ? kRight : kLeft;
        lastX = x;
        lastY = y;
        if (lastDir == kRight || should == kRight) {
          if (x == (uint32_t)W - 1 || y == 0 || y == (uint32_t)H - 1) break;
          const int g1 = gv(idx - W + 1), g2 = gv(idx + 1), g3 = gv(idx + W + 1);
          if (g1 >= g2 && g1 >= g3) {
            x++;
            y--;
          } else if (g3 >= g2 && g3 >= g1) {
            x++;
            y++;
          } else {
            x++;
          }
          lastDir = kRight;
        } else if (lastDir == kLeft || should == kLeft) {
          if (x == 0 || y == 0 || y == (uint32_t)H - 1) break;
          const int g1 = gv(idx - W - 1), g2 = gv(idx - 1), g3 = gv(idx + W - 1);
          if (g1 >= g2 && g1 >= g3) {
            x--;
            y--;
          } else if (g3 >= g2 && g3 >= g1) {
            x--;
            y++;
          } else {
            x--;
          }
          lastDir = kLeft;
        }
      } else {
        if (lastDir == kRight || lastDir == kLeft) should = y > lastY ? kDown : kUp;
        lastX = x;
        lastY = y;
        if (lastDir == kDown || should == kDown) {
          if (x == 0 || x == (uint32_t)W - 1 || y == (uint32_t)H - 1) break;
          const int g1 = gv(idx + W + 1), g2 = gv(idx + W), g3 = gv(idx + W - 1);
          if (g1 >= g2 && g1 >= g3) {
            x++;
            y++;
          } else if (g3 >= g2 && g3 >= g1) {
            x--;
            y++;
          } else {
            y++;
          }
          lastDir = kDown;
        } else if (lastDir == kUp || should == kUp) {
          if (x == 0 || x == (uint32_t)W - 1 || y == 0) break;
          const int g1 = gv(idx - W + 1), g2 = gv(idx - W), g3 = gv(idx - W - 1);
          if (g1 >= g2 && g1 >= g3) {
            x++;
            y--;
          } else if (g3 >= g2 && g3 >= g1) {
            x--;
            y--;
          } else {
            y--;
          }
          lastDir = kUp;
        }
      }
      idx = (int)(y * W + x);
    }
    return true;
  };
  for (size_t i = 0; i < ax.size(); i++) {
    const uint32_t x = ax[i], y = ay[i];
    const int idx = (int)(y * W + x);
    if (edge[idx]) continue;
    if (offPS > maxNumOfEdge) return -1;
    fS[offPS] = offF;
    const bool horiz = pd[idx] == kHorizontal;
    if (!walk(x, y, horiz ? kRight : kDown, fX, fY, offF)) return -1;
    edge[idx] = 0;  // the anchor is walked again by the second part
    sS[offPS] = offS;
    if (!walk(x, y, horiz ? kLeft : kUp, sX, sY, offS)) return -1;
    const int lenF = (int)(offF - fS[offPS]), lenS = (int)(offS - sS[offPS]);
    if (lenF + lenS < P.min_line_len + 1) {  // short edge, dropped (its pixels stay marked)
      offF = fS[offPS];
      offS = sS[offPS];
    } else {
      offPS++;
    }
  }
  if (offPS > maxNumOfEdge) return -1;
  fS[offPS] = offF;
  sS[offPS] = offS;
  E.x.clear();
  E.y.clear();
  E.sid.clear();
  for (uint32_t e = 0; e < offPS; e++) {
    E.sid.push_back((uint32_t)E.x.size());
    for (int t = (int)fS[e + 1] - 1; t >= (int)fS[e]; t--) {
      E.x.push_back(fX[t]);
      E.y.push_back(fY[t]);
    }
    for (uint32_t t = sS[e] + 1; t < sS[e + 1]; t++) {
      E.x.push_back(sX[t]);
      E.y.push_back(sY[t]);
    }
  }
  E.sid.push_back((uint32_t)E.x.size());
  return 1;
}

// The 2x2 normal equations of LeastSquaresLineFit_: ATA / ATV are float matrices whose
// entries are sums of integer products accumulated in double by cv::gemm
// (GEMMSingleMul<float, double>) and rounded to float once; the extension adds such
// a block to the running float matrices (ATA = ATA + tempMat).
struct Fit {
  float ata[4], atv[2];
};
void fit_block(const uint32_t* u, const uint32_t* v, uint32_t s, uint32_t e, float* ata, float* atv) {
  double s00 = 0, s01 = 0, s11 = 0, t0 = 0, t1 = 0;
  for (uint32_t i = s; i < e; i++) {
    const double a = (double)(float)u[i], b = (double)(float)v[i];
    s00 += a * a;
    s01 += a;
    s11 += 1.0;
    t0 += a * b;
    t1 += b;
  }
  ata[0] = (float)s00;
  ata[1] = (float)s01;
  ata[2] = (float)s01;
  ata[3] = (float)s11;
  atv[0] = (float)t0;
  atv[1] = (float)t1;
}
void solve(const Fit& F, double* le) {
  const double coef = 1.0 / ((double)F.ata[0] * (double)F.ata[3] - (double)F.ata[1] * (double)F.ata[2]);
  le[0] = coef * ((double)F.ata[3] * (double)F.atv[0] - (double)F.ata[1] * (double)F.atv[1]);
  le[1] = coef * ((double)F.ata[0] * (double)F.atv[1] - (double)F.ata[2] * (double)F.atv[0]);
}

struct Line {
  float ep[4];
  float direction;
};

// EDline(image, lines), binary_descriptor.cpp:2383-2630, with LineValidation_ (:2793-2874)
int edline(const Maps& M, const Chains& E, std::vector<Line>& out, const EdParams& P = kDefaultParams) {
  const int W = M.w, H = M.h;
  out.clear();
  const uint32_t nEdges = (uint32_t)E.sid.size() - 1;
  if (nEdges == 0) return 0;
  const double logNT = 2.0 * (std::log10((double)W) + std::log10((double)H));
  const uint32_t* ex = E.x.data();
  const uint32_t* ey = E.y.data();
  std::vector<uint32_t> lx(E.x.size() + 1), ly(E.y.size() + 1);
  uint32_t offL = 0, lineStart = 0, newOffS = 0;
  auto dirAt = [&](uint32_t x, uint32_t y) { return M.dir[(size_t)y * W + x]; };
  for (uint32_t e = 0; e < nEdges; e++) {
    uint32_t s = E.sid[e];
    const uint32_t end = E.sid[e + 1];
    double lineEq[2] = {0, 0};
    Fit F{};
    while (end > s + P.min_line_len) {
      double fitErr = 0;
      while (end > s + P.min_line_len) {  // an initial segment of minLineLen_ pixels
        const bool horiz = dirAt(ex[s], ey[s]) == kHorizontal;
        const uint32_t* u = horiz ? ex : ey;
        const uint32_t* v = horiz ? ey : ex;
        fit_block(u, v, s, s + P.min_line_len, F.ata, F.atv);
        solve(F, lineEq);
        double err = 0;
        for (uint32_t i = s; i < s + P.min_line_len; i++) {
          const double c = (double)v[i] - (double)u[i] * lineEq[0] - lineEq[1];
          err += c * c;
        }
        fitErr = std::sqrt(err);
        if (fitErr <= P.fit_err_th) break;
        s += kSkip;
      }
      if (fitErr > P.fit_err_th) break;
      lineStart = offL;
      const bool horiz = dirAt(ex[s], ey[s]) == kHorizontal;
      double coef1 = 0;
      bool extended = true, first = true;
      int tryTimes = 0, outliers = 0;
      while (extended) {
        tryTimes++;
        if (first) {
          first = false;
          for (int i = 0; i < P.min_line_len; i++) {
            lx[offL] = ex[s];
            ly[offL++] = ey[s++];
          }
        } else {  // LeastSquaresLineFit_(..., newOffsetS, offsetInLineArray): add the new block
          const bool h0 = dirAt(lx[lineStart], ly[lineStart]) == kHorizontal;
          Fit T{};
          fit_block(h0 ? lx.data() : ly.data(), h0 ? ly.data() : lx.data(), newOffS, offL, T.ata, T.atv);
          for (int q = 0; q < 4; q++) F.ata[q] = F.ata[q] + T.ata[q];
          for (int q = 0; q < 2; q++) F.atv[q] = F.atv[q] + T.atv[q];
          solve(F, lineEq);
        }
        coef1 = 1 / std::sqrt(horiz ? lineEq[0] * lineEq[0] + 1 : 1 + lineEq[0] * lineEq[0]);
        outliers = 0;
        newOffS = offL;
        while (end > s) {
          const double d = horiz ? std::fabs(lineEq[0] * ex[s] - ey[s] + lineEq[1]) * coef1
                                 : std::fabs(ex[s] - lineEq[0] * ey[s] - lineEq[1]) * coef1;
          lx[offL] = ex[s];
          ly[offL++] = ey[s++];
          if (d > P.fit_err_th) {
            if (++outliers > 3) break;
          } else {
            outliers = 0;
          }
        }
        offL -= outliers;
        s -= outliers;
        extended = offL - newOffS > 0 && tryTimes < kTryTime;
      }
      double le[3];
      if (horiz) {
        le[0] = lineEq[0] * coef1;
        le[1] = -1 * coef1;
        le[2] = lineEq[1] * coef1;
      } else {
        le[0] = 1 * coef1;
        le[1] = -lineEq[0] * coef1;
        le[2] = -lineEq[1] * coef1;
      }
      // LineValidation_
      bool ok = false;
      float direction = 0;
      {
        const int n = (int)(offL - lineStart);
        int mgx = 0, mgy = 0;
        std::vector<double> pdir(n);
        for (int i = 0; i < n; i++) {
          const size_t idx = (size_t)ly[lineStart + i] * W + lx[lineStart + i];
          mgx += M.dx[idx];
          mgy += M.dy[idx];
          pdir[i] = std::atan2(-(double)M.dx[idx], (double)M.dy[idx]);
        }
        const double dxl = std::fabs(le[1]), dyl = std::fabs(le[0]);
        bool reject = mgx == 0 && mgy == 0;
        if (!reject) {
          if (mgx > 0 && mgy >= 0) direction = (float)std::atan2(-dyl, dxl);
          if (mgx <= 0 && mgy > 0) direction = (float)std::atan2(dyl, dxl);
          if (mgx < 0 && mgy <= 0) direction = (float)std::atan2(dyl, -dxl);
          if (mgx >= 0 && mgy < 0) direction = (float)std::atan2(-dyl, -dxl);
          if (std::fabs(direction) < 0.15 || M_PI - std::fabs(direction) < 0.15)
            if (std::fabs(le[2]) < 10 || std::fabs(H - std::fabs(le[2])) < 10) reject = true;
          if (std::fabs(std::fabs(direction) - M_PI * 0.5) < 0.15)
            if (std::fabs(le[2]) < 10 || std::fabs(W - std::fabs(le[2])) < 10) reject = true;
        }
        if (!P.validate) {
          ok = true;
        } else if (!reject) {
          int k = 0;
          for (int i = 0; i < n; i++) {
            const double dd = std::fabs(direction - pdir[i]);
            if (std::fabs(2 * M_PI - dd) < 0.392699 || dd < 0.392699) k++;
          }
          ok = nfa(n, k, 0.125, logNT) > 0;
        }
      }
      if (ok) {
        const double a1 = le[1] * le[1], a2 = le[0] * le[0], a3 = le[0] * le[1], a4 = le[2] * le[0],
                     a5 = le[2] * le[1];
        Line L;
        uint32_t Px = lx[lineStart], Py = ly[lineStart];
        L.ep[0] = (float)(a1 * Px - a3 * Py - a4);
        L.ep[1] = (float)(a2 * Py - a3 * Px - a5);
        Px = lx[offL - 1];
        Py = ly[offL - 1];
        L.ep[2] = (float)(a1 * Px - a3 * Py - a4);
        L.ep[3] = (float)(a2 * Py - a3 * Px - a5);
        L.direction = direction;
        out.push_back(L);
      } else {
        offL = lineStart;
      }
    }
  }
  return 1;
}

}  // namespace

extern "C" {

int orc_line_maps(const uint8_t* gray, int w, int h, uint8_t* blur, int16_t* dx, int16_t* dy, int16_t* g,
                  uint8_t* dir) {
  Maps M;
  compute_maps(gray, w, h, M);
  const size_t n = (size_t)w * h;
  if (blur) std::memcpy(blur, M.blur.data(), n);
  if (dx) std::memcpy(dx, M.dx.data(), n * 2);
  if (dy) std::memcpy(dy, M.dy.data(), n * 2);
  if (g) std::memcpy(g, M.g.data(), n * 2);
  if (dir) std::memcpy(dir, M.dir.data(), n);
  return 0;
}

// edge chains of EdgeDrawing: pixel (x, y) pairs concatenated, sid[numOfEdges + 1]
int orc_edge_chains(const uint8_t* gray, int w, int h, uint32_t* xy, int cap_px, uint32_t* sid, int cap_edges,
                    int* n_px, int* n_edges) {
  Maps M;
  compute_maps(gray, w, h, M);
  Chains E;
  if (edge_drawing(M, E, nullptr) != 1) return -1;
  *n_px = (int)E.x.size();
  *n_edges = (int)E.sid.size() - 1;
  for (int i = 0; i < std::min(*n_px, cap_px); i++) {
    xy[2 * i] = E.x[i];
    xy[2 * i + 1] = E.y[i];
  }
  for (int i = 0; i < std::min(*n_edges + 1, cap_edges + 1); i++) sid[i] = E.sid[i];
  return 0;
}

// The restatement under other knobs, for its pinning against the Edge Drawing library's own
// outputs (Thirdparty/EDTest/ED-EdgeMap.pgm, EDLinesTest/LineSegments.txt):
// ip = {gradient threshold, anchor threshold, scan interval, min line length, gdiv, validate}.
static EdParams ed_params(const int* ip, double fit_err) {
  EdParams P;
  P.grad_th = ip[0];
  P.anchor_th = ip[1];
  P.scan = ip[2];
  P.min_line_len = ip[3];
  P.gdiv = ip[4];
  P.fit_err_th = fit_err;
  P.validate = ip[5];
  return P;
}
// the kept edge chains' pixels as a 255 / 0 map (EDTest/main.cpp:65-72 draws ED's segments so)
int orc_ed_edge_map(const uint8_t* gray, int w, int h, const int* ip, double fit_err, uint8_t* map, int* n_chains) {
  const EdParams P = ed_params(ip, fit_err);
  Maps M;
  compute_maps(gray, w, h, M, P);
  Chains E;
  if (edge_drawing(M, E, nullptr, P) != 1) return -1;
  std::memset(map, 0, (size_t)w * h);
  for (size_t i = 0; i < E.x.size(); i++) map[(size_t)E.y[i] * w + E.x[i]] = 255;
  *n_chains = (int)E.sid.size() - 1;
  return 0;
}
// EDline's segments (endpoints x1, y1, x2, y2 as fitted, no length filter or reordering)
int orc_ed_segments(const uint8_t* gray, int w, int h, const int* ip, double fit_err, float* out, int cap,
                    int* n_out) {
  const EdParams P = ed_params(ip, fit_err);
  Maps M;
  compute_maps(gray, w, h, M, P);
  Chains E;
  if (edge_drawing(M, E, nullptr, P) != 1) return -1;
  std::vector<Line> L;
  edline(M, E, L, P);
  *n_out = (int)L.size();
  for (int i = 0; i < std::min(*n_out, cap); i++) std::memcpy(out + 4 * (size_t)i, L[i].ep, sizeof(float) * 4);
  return *n_out > cap ? -2 : 0;
}

// detect_raw_lines (octave 0) + filter_lines(length > min_length) + keylines_to_mat:
// per kept line (startX, startY, endX, endY, angle, lineLength), in EDline order
int orc_edlines(const uint8_t* gray, int w, int h, float min_length, float* out, int cap, int* n_out) {
  Maps M;
  compute_maps(gray, w, h, M);
  Chains E;
  if (edge_drawing(M, E, nullptr) != 1) return -1;
  std::vector<Line> L;
  edline(M, E, L);
  int n = 0;
  for (const Line& l : L) {
    // OctaveKeyLines, binary_descriptor.cpp:866-887, 1073-1141 (scale 1)
    const float dxa = std::fabs(l.ep[0] - l.ep[2]), dya = std::fabs(l.ep[1] - l.ep[3]);
    const float length = std::sqrt(dxa * dxa + dya * dya);
    const float s1 = l.ep[0], s2 = l.ep[1], e1 = l.ep[2], e2 = l.ep[3];
    const float ddx = e1 - s1, ddy = e2 - s2, d = l.direction;
    bool change = false;
    if (d >= -0.75 * M_PI && d < -0.25 * M_PI && ddy > 0) change = true;
    if (d >= -0.25 * M_PI && d < 0.25 * M_PI && ddx < 0) change = true;
    if (d >= 0.25 * M_PI && d < 0.75 * M_PI && ddy < 0) change = true;
    if (((d >= 0.75 * M_PI && d < M_PI) || (d >= -M_PI && d < -0.75 * M_PI)) && ddx > 0) change = true;
    if (!(length > min_length)) continue;  // filter_lines, line_lbd_allclass.cpp:205-213
    if (n < cap) {
      float* o = out + 6 * (size_t)n;
      o[0] = change ? e1 : s1;
      o[1] = change ? e2 : s2;
      o[2] = change ? s1 : e1;
      o[3] = change ? s2 : e2;
      o[4] = d;
      o[5] = length;
    }
    n++;
  }
  *n_out = n;
  return n > cap ? -2 : 0;
}

// BinaryDescriptor::detectImpl's input conversion (src/line_detect/libs/binary_descriptor.cpp:490-495):
// a frame with channels != 1 -- the colour rawImage of the EAO Frame ctor (src/Frame.cc:324,
// src/Tracking.cc:340,389) -- is converted with COLOR_BGR2GRAY whatever Camera.RGB says (so not
// the tracker's mImGray when mbRGB): OpenCV 3.2 RGB2Gray<uchar> in the BGR coefficient
// order, orb_ref.cpp's orc_color_to_gray with rgb = 0. Then orc_edlines on that gray.
int orc_edlines_color(const uint8_t* img, int w, int h, int pitch, int cn, float min_length, float* out, int cap,
                      int* n_out) {
  std::vector<uint8_t> gray((size_t)w * h);
  if (cn == 1) {
    for (int y = 0; y < h; y++) std::memcpy(&gray[(size_t)y * w], img + (size_t)y * pitch, w);
  } else if (cn == 3 || cn == 4) {
    orc_color_to_gray(img, w, h, pitch, cn, 0, gray.data());
  } else {
    return -3;
  }
  return orc_edlines(gray.data(), w, h, min_length, out, cap, n_out);
}

}  // extern "C"
