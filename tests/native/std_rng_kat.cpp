// std_rng_kat.cpp -- TEST INFRASTRUCTURE. The random streams the reference
// relies on, produced by THIS toolchain's libstdc++ (<random>, std::shuffle,
// std::sort), so tests/test_oracle_kat.py can pin the oracle's hand-coded
// restatement (oracle/iforest_ref.h) against the library itself. Own code:
// a textbook isolation forest written against the std:: API with the call
// pattern SURVEY.md §8c describes for include/isolation_forest.h.
//
// usage: std_rng_kat MODE ARGS...   writes little-endian binary to stdout
//   mt SEED N              N raw mt19937 outputs (uint32)
//   lemire SEED N RANGE    N draws of uniform_int_distribution<uint32_t>(0, RANGE-1)
//   shuffle SEED N         std::shuffle of 0..N-1 (uint32)
//   real SEED N LO HI      N draws of uniform_real_distribution<float>(LO, HI)
//   iforest N TREES SEED SAMPLE   reads N*3 float32 from stdin, writes N float64
//   sort5 N                reads N*5 float32 rows, std::sort by row[1] descending (the
//                          Tracking.cc:64-68 VIC comparator), writes the sorted rows
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <vector>

typedef std::array<float, 3> Item;

static double c_of(uint32_t n) {
  if (n > 2) {
    const double h = std::log((double)(n - 1)) + 0.5772156649;
    return 2.0 * h - (2.0 * (n - 1)) / (double)n;
  }
  return n == 2 ? 1.0 : 0.0;
}

struct Node {
  uint32_t dim = 0, size = 0;
  float split = 0;
  std::unique_ptr<Node> l, r;
  bool build(std::mt19937& g, std::vector<Item*>& d, uint32_t first, uint32_t last, uint32_t depth,
             uint32_t maxd) {
    if (last < first || last >= d.size()) return false;
    if (last - first < 1 || depth >= maxd) {
      size = last - first + 1;
      return true;
    }
    std::uniform_int_distribution<uint32_t> dd(0, 2);
    dim = dd(g);
    const uint32_t k = dim;
    std::sort(d.begin() + first, d.begin() + last + 1, [k](const Item* a, const Item* b) { return (*a)[k] < (*b)[k]; });
    const float mn = (*d[first])[k], mx = (*d[last])[k];
    if (mn == mx) {
      size = last - first + 1;
      return true;
    }
    std::uniform_real_distribution<float> u(mn, mx);
    split = u(g);
    uint32_t mid = first;
    for (; mid <= last; mid++)
      if ((*d[mid])[k] >= split) break;
    if (mid == first) {
      size = last - first + 1;
      return true;
    }
    l.reset(new Node());
    r.reset(new Node());
    return l->build(g, d, first, mid - 1, depth + 1, maxd) && r->build(g, d, mid, last, depth + 1, maxd);
  }
  double path(const Item& x, uint32_t depth) const {
    if (!l || !r) return depth + c_of(size);
    return x[dim] < split ? l->path(x, depth + 1) : r->path(x, depth + 1);
  }
};

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const char* m = argv[1];
  if (!std::strcmp(m, "mt")) {
    std::mt19937 g((uint32_t)std::strtoul(argv[2], 0, 10));
    const int n = std::atoi(argv[3]);
    for (int i = 0; i < n; i++) {
      uint32_t v = g();
      std::fwrite(&v, 4, 1, stdout);
    }
  } else if (!std::strcmp(m, "lemire")) {
    std::mt19937 g((uint32_t)std::strtoul(argv[2], 0, 10));
    const int n = std::atoi(argv[3]);
    std::uniform_int_distribution<uint32_t> d(0, (uint32_t)std::strtoul(argv[4], 0, 10) - 1);
    for (int i = 0; i < n; i++) {
      uint32_t v = d(g);
      std::fwrite(&v, 4, 1, stdout);
    }
  } else if (!std::strcmp(m, "shuffle")) {
    std::mt19937 g((uint32_t)std::strtoul(argv[2], 0, 10));
    std::vector<uint32_t> v(std::atoi(argv[3]));
    for (size_t i = 0; i < v.size(); i++) v[i] = (uint32_t)i;
    std::shuffle(v.begin(), v.end(), g);
    std::fwrite(v.data(), 4, v.size(), stdout);
  } else if (!std::strcmp(m, "real")) {
    std::mt19937 g((uint32_t)std::strtoul(argv[2], 0, 10));
    const int n = std::atoi(argv[3]);
    std::uniform_real_distribution<float> d((float)std::atof(argv[4]), (float)std::atof(argv[5]));
    for (int i = 0; i < n; i++) {
      float v = d(g);
      std::fwrite(&v, 4, 1, stdout);
    }
  } else if (!std::strcmp(m, "iforest")) {
    const uint32_t n = std::atoi(argv[2]), trees = std::atoi(argv[3]), seed = std::strtoul(argv[4], 0, 10),
                   sample = std::atoi(argv[5]);
    std::vector<Item> data(n);
    for (auto& it : data)
      if (std::fread(it.data(), 4, 3, stdin) != 3) return 3;
    std::mt19937 gen(seed);
    std::uniform_int_distribution<uint32_t> ud(0, 0xffffffffu);
    std::vector<std::unique_ptr<Node>> roots(trees);
    for (uint32_t t = 0; t < trees; t++) {
      std::mt19937 tg(ud(gen));
      std::vector<uint32_t> ids(n);
      for (uint32_t i = 0; i < n; i++) ids[i] = i;
      std::shuffle(ids.begin(), ids.end(), tg);
      std::vector<Item*> local(sample);
      for (uint32_t i = 0; i < sample; i++) local[i] = &data[ids[i]];
      roots[t].reset(new Node());
      if (!roots[t]->build(tg, local, 0, sample - 1, 0, (uint32_t)std::ceil(std::log2((double)sample)))) return 4;
    }
    const double c = c_of(sample);
    for (uint32_t i = 0; i < n; i++) {
      double tot = 0;
      for (auto& r : roots) tot += r->path(data[i], 0);
      const double s = std::pow(2.0, -(tot / (double)trees) / c);
      std::fwrite(&s, 8, 1, stdout);
    }
  } else if (!std::strcmp(m, "sort5")) {
    std::vector<std::array<float, 5>> rows(std::atoi(argv[2]));
    for (auto& r : rows)
      if (std::fread(r.data(), 4, 5, stdin) != 5) return 3;
    std::sort(rows.begin(), rows.end(),
              [](const std::array<float, 5>& a, const std::array<float, 5>& b) { return a[1] > b[1]; });
    for (auto& r : rows) std::fwrite(r.data(), 4, 5, stdout);
  } else {
    return 2;
  }
  return 0;
}
