/*
 * iforest_ref.h -- explicit restatement of include/isolation_forest.h with the
 * random streams of libstdc++ 11 (GCC 11.4, this container) coded out by hand
 * so the result does not depend on the host toolchain:
 *   std::mt19937                                  (standard recurrence)
 *   uniform_int_distribution, 32-bit URNG         (Lemire nearly-divisionless,
 *                                                  uniform_int_dist.h:240-317)
 *   std::shuffle                                  (paired draws when n*n <= 2^32-1,
 *                                                  stl_algo.h:3706-3790)
 *   generate_canonical<float,24> / uniform_real   (random.tcc:3348-3373,
 *                                                  random.h:1870)
 * TEST INFRASTRUCTURE ONLY.
 */
#ifndef EAO_IFOREST_REF_H
#define EAO_IFOREST_REF_H
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <memory>
#include <vector>

namespace orc {

struct MT19937 {
  uint32_t mt[624];
  int idx;
  explicit MT19937(uint32_t s) { seed(s); }
  void seed(uint32_t s) {
    mt[0] = s;
    for (int i = 1; i < 624; i++) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    idx = 624;
  }
  void twist() {
    for (int k = 0; k < 624; k++) {
      uint32_t y = (mt[k] & 0x80000000u) | (mt[(k + 1) % 624] & 0x7fffffffu);
      mt[k] = mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    idx = 0;
  }
  uint32_t operator()() {
    if (idx >= 624) twist();
    uint32_t y = mt[idx++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
};

// uniform_int_distribution downscaling with a 32-bit URNG: [0, range)
inline uint32_t lemire(MT19937& g, uint32_t range) {
  uint64_t product = (uint64_t)g() * (uint64_t)range;
  uint32_t low = (uint32_t)product;
  if (low < range) {
    uint32_t threshold = (uint32_t)(0u - range) % range;
    while (low < threshold) {
      product = (uint64_t)g() * (uint64_t)range;
      low = (uint32_t)product;
    }
  }
  return (uint32_t)(product >> 32);
}

inline void shuffle_ids(std::vector<uint32_t>& v, MT19937& g) {
  const uint64_t n = v.size();
  if (n == 0) return;
  const uint64_t urngrange = 0xffffffffull;
  if (urngrange / n >= n) {
    uint64_t i = 1;
    if ((n % 2) == 0) {
      uint32_t pos = lemire(g, 2);
      std::swap(v[i], v[pos]);
      i++;
    }
    while (i != n) {
      const uint64_t swap_range = i + 1;
      uint32_t x = lemire(g, (uint32_t)(swap_range * (swap_range + 1)));
      uint64_t p1 = x / (swap_range + 1), p2 = x % (swap_range + 1);
      std::swap(v[i], v[p1]);
      i++;
      std::swap(v[i], v[p2]);
      i++;
    }
    return;
  }
  for (uint64_t i = 1; i < n; i++) std::swap(v[i], v[lemire(g, (uint32_t)(i + 1))]);
}

inline float canonical_float(MT19937& g) {
  float sum = (float)g() * 1.0f;
  float tmp = 4294967296.0f;
  float ret = sum / tmp;
  if (ret >= 1.0f) ret = std::nextafter(1.0f, 0.0f);
  return ret;
}

inline float uniform_real(MT19937& g, float a, float b) { return canonical_float(g) * (b - a) + a; }

// CalculateC / CalculateH, isolation_forest.h:97-118
inline double iforest_c(uint32_t n) {
  if (n > 2) {
    double h = std::log((double)(n - 1)) + 0.5772156649;
    return double(2.0 * h) - (double(2.0 * (n - 1)) / double(n));
  } else if (n == 2)
    return 1.0;
  return 0.0;
}

struct IFNode {
  uint32_t dim = 0;
  float split = 0.f;
  uint32_t size = 0;
  std::unique_ptr<IFNode> left, right;
  bool leaf() const { return !left || !right; }
};

typedef float item3[3];

// Node::Build, isolation_forest.h:165-224
inline bool if_build(IFNode& nd, MT19937& rng, std::vector<const float*>& data, uint32_t first,
                     uint32_t last, uint32_t depth, uint32_t maxDepth) {
  if (last < first || last >= data.size()) return false;
  if (last - first < 1 || depth >= maxDepth) {
    nd.size = (last - first) + 1;
    return true;
  }
  uint32_t dim = nd.dim = lemire(rng, 3);
  std::sort(data.begin() + first, data.begin() + last + 1,
            [dim](const float* l, const float* r) { return l[dim] < r[dim]; });
  float minV = data[first][dim], maxV = data[last][dim];
  if (minV == maxV) {
    nd.size = (last - first) + 1;
    return true;
  }
  nd.split = uniform_real(rng, minV, maxV);
  uint32_t middle = first;
  for (middle = first; middle <= last; middle++)
    if (data[middle][dim] >= nd.split) break;
  if (middle == first) {
    nd.size = (last - first) + 1;
    return true;
  }
  nd.left.reset(new IFNode());
  nd.right.reset(new IFNode());
  if (!if_build(*nd.left, rng, data, first, middle - 1, depth + 1, maxDepth)) return false;
  if (!if_build(*nd.right, rng, data, middle, last, depth + 1, maxDepth)) return false;
  return true;
}

inline double if_path(const IFNode& nd, const float* x, uint32_t depth) {
  if (nd.leaf()) return double(depth) + iforest_c(nd.size);
  if (x[nd.dim] < nd.split) return if_path(*nd.left, x, depth + 1);
  return if_path(*nd.right, x, depth + 1);
}

// IsolationForest::Build + GetAnomalyScores (isolation_forest.h:448-530)
inline bool iforest_scores(const float* pts, uint32_t n, uint32_t trees, uint32_t seed,
                           uint32_t sampleSize, std::vector<double>& scores) {
  if (!n || !sampleSize || sampleSize > n) return false;
  MT19937 gen(seed);
  std::vector<std::unique_ptr<IFNode>> roots(trees);
  for (uint32_t t = 0; t < trees; t++) {
    uint32_t tseed = gen();  // uniform_int<uint32>(0, UINT32_MAX): raw draw
    MT19937 tg(tseed);
    std::vector<uint32_t> ids(n);
    for (uint32_t i = 0; i < n; i++) ids[i] = i;
    shuffle_ids(ids, tg);
    std::vector<const float*> local(sampleSize);
    for (uint32_t i = 0; i < sampleSize; i++) local[i] = pts + 3 * (size_t)ids[i];
    uint32_t maxDepth = (uint32_t)std::ceil(std::log2((double)sampleSize));
    roots[t].reset(new IFNode());
    if (!if_build(*roots[t], tg, local, 0, sampleSize - 1, 0, maxDepth)) return false;
  }
  const double c = iforest_c(sampleSize);
  scores.resize(n);
  for (uint32_t i = 0; i < n; i++) {
    double total = 0;
    for (uint32_t t = 0; t < trees; t++) total += if_path(*roots[t], pts + 3 * (size_t)i, 0);
    double avg = total / double(trees);
    scores[i] = std::pow(2.0, -avg / c);
  }
  return true;
}

}  // namespace orc
#endif
