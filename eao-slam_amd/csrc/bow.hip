// bow.hip -- the bag-of-words path of tracking on gfx950:
//   Frame::ComputeBoW (src/Frame.cc:516-523) = DBoW2 TemplatedVocabulary::transform(desc,
//     BowVector, FeatureVector, levelsup 4) for the ORB vocabulary (TF_IDF weights, L1 norm)
//     (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1139-1206,1230-1271);
//   ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&) (src/ORBmatcher.cc:159-288).
//
// Kernels:
//   k_bow_words   one thread per (frame, feature): the feature descends the vocabulary tree
//                 (children CSR in HBM, 32-byte node descriptors, first-minimum Hamming child
//                 per level), giving its word, weight and the node at level L - levelsup;
//   k_bow_build   one 1024-thread workgroup per frame: the (node, feature) and (word, feature)
//                 keys are bitonic-sorted in LDS; node runs give the FeatureVector CSR (features
//                 ascending within a node, nodes ascending = std::map order), word runs give the
//                 BowVector (weights summed in feature order = addWeight's order, then the L1
//                 norm summed in word order and divided out, as BowVector::normalize);
//   k_bow_search  one wave per keyframe node: the frame node with the same id is found by binary
//                 search (the reference's merge walk visits exactly the common ids, and a feature
//                 sits in one node only, so nodes are independent); the node's keyframe features
//                 are resolved in order against the frame features still free (LDS flags), each
//                 lane holding a strided share: (best, first index, second best) merged across
//                 the wave; ratio test, TH_LOW;
//   k_bow_rot     one workgroup per search: rotation histogram, ComputeThreeMaxima, removal.
// Every result is integer / exact (the weights are sums of the vocabulary's doubles in the
// reference's order), so the bar is bit-exact against oracle/bow_ref.cpp.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstring>
#include <string>
#include <vector>

#include "../../include/eao_accel.h"
#include "common.h"
#include "orb.h"

namespace eao {
namespace {

constexpr int TH_LOW = 50, HISTO_LENGTH = 30;  // ORBmatcher.cc:37-39
constexpr int BOW_MAXN = 4096;                 // features per frame of k_bow_build (LDS sort)
constexpr int NODE_MAXF = 1024;                // frame features per vocabulary node (search flags)

__device__ __forceinline__ int ham32(const uint8_t* a, uint4 b0, uint4 b1) {
  const uint4 a0 = *(const uint4*)a, a1 = *(const uint4*)(a + 16);
  return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
         __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

struct VocabDev {
  const uint8_t* desc;      // [n][32]
  const int* child_start;   // [n + 1]
  const int* child_ids;     // children of node k: child_ids[child_start[k] .. child_start[k+1])
  const int* word;          // [n] (-1 inner)
  const double* weight;     // [n]
  int L, empty;
};

// TemplatedVocabulary::transform(feature, word_id, weight, &nid, levelsup)
__global__ __launch_bounds__(256) void k_bow_words(VocabDev V, int cap, const int* __restrict__ counts,
                                                   const uint8_t* __restrict__ desc, int levelsup,
                                                   int* __restrict__ fword, double* __restrict__ fweight,
                                                   int* __restrict__ fnode) {
  const int f = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
  if (i >= min(counts[f], cap)) return;
  const size_t o = (size_t)f * cap + i;
  if (V.empty) {
    fword[o] = -1;
    fweight[o] = 0.0;
    fnode[o] = 0;
    return;
  }
  const uint8_t* d = desc + 32 * o;
  const uint4 b0 = *(const uint4*)d, b1 = *(const uint4*)(d + 16);
  const int nid_level = V.L - levelsup;
  int nid = 0, fid = 0, level = 0;
  do {
    ++level;
    const int c0 = V.child_start[fid], c1 = V.child_start[fid + 1];
    fid = V.child_ids[c0];
    int best = ham32(V.desc + 32 * (size_t)fid, b0, b1);
    for (int c = c0 + 1; c < c1; c++) {
      const int id = V.child_ids[c];
      const int dd = ham32(V.desc + 32 * (size_t)id, b0, b1);
      if (dd < best) {
        best = dd;
        fid = id;
      }
    }
    if (level == nid_level) nid = fid;
  } while (V.child_start[fid + 1] > V.child_start[fid]);
  const double w = V.weight[fid];
  fword[o] = w > 0 ? V.word[fid] : -1;  // stopped words are not added
  fweight[o] = w;
  fnode[o] = nid;
}

// bitonic sort of N (power of two) u64 keys in LDS by the whole block
template <int T>
__device__ void lds_sort(unsigned long long* k, int N) {
  for (int size = 2; size <= N; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int t = threadIdx.x; t < (N >> 1); t += T) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const unsigned long long a = k[lo], b = k[hi];
        if ((a > b) == up) {
          k[lo] = b;
          k[hi] = a;
        }
      }
    }
  __syncthreads();
}

// block exclusive scan of one int per thread (T threads), returns the total
template <int T>
__device__ int block_excl_scan(int v, int& excl, int* s_w) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int inc = v;
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  int base = 0, tot = 0;
  for (int q = 0; q < T / 64; q++) {
    if (q < w) base += s_w[q];
    tot += s_w[q];
  }
  excl = base + inc - v;
  __syncthreads();
  return tot;
}

__global__ __launch_bounds__(1024) void k_bow_build(int cap, const int* __restrict__ counts,
                                                    const int* __restrict__ fword,
                                                    const double* __restrict__ fweight,
                                                    const int* __restrict__ fnode, int* __restrict__ word_ids,
                                                    double* __restrict__ word_w, int* __restrict__ n_words,
                                                    int* __restrict__ node_ids, int* __restrict__ node_start,
                                                    int* __restrict__ node_feats, int* __restrict__ n_nodes) {
  constexpr int T = 1024;
  __shared__ unsigned long long s_key[BOW_MAXN];
  __shared__ double s_sum[BOW_MAXN];
  __shared__ int s_w[T / 64];
  const int f = blockIdx.x, t = threadIdx.x;
  const int n = min(counts[f], cap);
  int N = 1;
  while (N < n) N <<= 1;
  const size_t o = (size_t)f * cap;
  int* NI = node_ids + o;
  int* NS = node_start + (size_t)f * (cap + 1);
  int* NF = node_feats + o;
  // ---- FeatureVector: (node, feature) keys of the not-stopped features
  for (int i = t; i < N; i += T)
    s_key[i] = (i < n && fword[o + i] >= 0) ? (((unsigned long long)fnode[o + i] << 13) | (unsigned long long)i)
                                            : ~0ull;
  lds_sort<T>(s_key, N);
  int nvalid_total = 0, nn_total = 0;
  for (int base = 0; base < N; base += T) {
    const int i = base + t;
    const unsigned long long k = i < N ? s_key[i] : ~0ull;
    const bool valid = k != ~0ull;
    const bool head = valid && (i == 0 || (s_key[i - 1] >> 13) != (k >> 13));
    int ex;
    const int tot = block_excl_scan<T>(head ? 1 : 0, ex, s_w);
    if (valid) NF[i] = (int)(k & 0x1fff);
    if (head) {
      NI[nn_total + ex] = (int)(k >> 13);
      NS[nn_total + ex] = i;
    }
    int exv;
    nvalid_total += block_excl_scan<T>(valid ? 1 : 0, exv, s_w);
    nn_total += tot;
  }
  if (t == 0) {
    NS[nn_total] = nvalid_total;
    n_nodes[f] = nn_total;
  }
  __syncthreads();
  // ---- BowVector: (word, feature) keys; weights summed per word in feature order
  for (int i = t; i < N; i += T)
    s_key[i] = (i < n && fword[o + i] >= 0) ? (((unsigned long long)fword[o + i] << 13) | (unsigned long long)i)
                                            : ~0ull;
  lds_sort<T>(s_key, N);
  int nw_total = 0;
  int* WI = word_ids + o;
  double* WW = word_w + o;
  for (int base = 0; base < N; base += T) {
    const int i = base + t;
    const unsigned long long k = i < N ? s_key[i] : ~0ull;
    const bool valid = k != ~0ull;
    const bool head = valid && (i == 0 || (s_key[i - 1] >> 13) != (k >> 13));
    int ex;
    const int tot = block_excl_scan<T>(head ? 1 : 0, ex, s_w);
    if (head) {
      double s = fweight[o + (k & 0x1fff)];
      for (int j = i + 1; j < N && (s_key[j] >> 13) == (k >> 13) && s_key[j] != ~0ull; j++)
        s += fweight[o + (s_key[j] & 0x1fff)];
      s_sum[nw_total + ex] = s;
      WI[nw_total + ex] = (int)(k >> 13);
    }
    nw_total += tot;
  }
  __syncthreads();
  __shared__ double s_norm;
  if (t == 0) {  // BowVector::normalize(L1): sum in word order
    double norm = 0.0;
    for (int j = 0; j < nw_total; j++) norm += fabs(s_sum[j]);
    s_norm = norm;
    n_words[f] = nw_total;
  }
  __syncthreads();
  const double norm = s_norm;
  for (int j = t; j < nw_total; j += T) WW[j] = norm > 0.0 ? s_sum[j] / norm : s_sum[j];
}

struct SearchSlot {
  const eao_keypoint_dev* kps;
  const uint8_t* desc;
  const uint8_t* valid;  // keyframe side only
  const int* nn;         // [nsearch] node counts
  const int* ids;        // [nsearch][cap]
  const int* start;      // [nsearch][cap + 1]
  const int* feats;      // [nsearch][cap]
};

// KFKF = false: SearchByBoW(KeyFrame*, Frame&) -- K the keyframe (outer), Fr the frame (inner),
//   match[iF] = ikf, distance bar <= TH_LOW (ORBmatcher.cc:159-288);
// KFKF = true: SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2) -- K = KF1 (outer), Fr = KF2 (inner, its map
//   points checked: Fr.valid), match12[idx1] = idx2, bar < TH_LOW (ORBmatcher.cc:522-655). The inner
//   side's taken flags are vbMatched2 there, the "already matched" test of the frame here.
template <bool KFKF>
__global__ __launch_bounds__(256) void k_bow_search(int cap, SearchSlot K, SearchSlot Fr, float nnratio,
                                                    int* __restrict__ f_match, int* __restrict__ err) {
  __shared__ uint8_t s_flag[4][NODE_MAXF];
  const int s = blockIdx.y, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int j = blockIdx.x * 4 + w;
  if (j >= K.nn[s]) return;
  const size_t so = (size_t)s * cap, ss = (size_t)s * (cap + 1);
  const int id = K.ids[so + j];
  // lower_bound over the frame's node ids
  int lo = 0, hi = Fr.nn[s];
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (Fr.ids[so + mid] < id) lo = mid + 1;
    else hi = mid;
  }
  if (lo >= Fr.nn[s] || Fr.ids[so + lo] != id) return;
  const int q0 = Fr.start[ss + lo], nq = Fr.start[ss + lo + 1] - q0;
  if (nq > NODE_MAXF) {  // reported per search through nmatches (k_bow_rot)
    if (lane == 0) atomicOr(&err[s], 1);
    return;
  }
  uint8_t* flag = s_flag[w];
  for (int q = lane; q < nq; q += 64)
    flag[q] = KFKF ? (Fr.valid[so + Fr.feats[so + q0 + q]] ? 0 : 1) : 0;  // !pMP2 || isBad(): never taken
  const int p0 = K.start[ss + j], p1 = K.start[ss + j + 1];
  int* M = f_match + so;
  for (int p = p0; p < p1; p++) {
    const int ikf = K.feats[so + p];
    if (!K.valid[so + ikf]) continue;  // !pMP || pMP->isBad()
    const uint8_t* dk = K.desc + 32 * (so + ikf);
    const uint4 b0 = *(const uint4*)dk, b1 = *(const uint4*)(dk + 16);
    // per lane: best distance, its first position, second best (the reference's scan order
    // restricted to the lane's positions), then merged across the wave
    int d1 = 256, p1 = 0x7fffffff, d2 = 256;
    for (int q = lane; q < nq; q += 64) {
      if (flag[q]) continue;
      const int iF = Fr.feats[so + q0 + q];
      const int d = ham32(Fr.desc + 32 * (so + iF), b0, b1);
      if (d < d1) {
        d2 = d1;
        d1 = d;
        p1 = q;
      } else if (d < d2) {
        d2 = d;
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const int od1 = __shfl_xor(d1, o, 64), op1 = __shfl_xor(p1, o, 64), od2 = __shfl_xor(d2, o, 64);
      if (od1 < d1 || (od1 == d1 && op1 < p1)) {
        d2 = min(od2, d1);
        d1 = od1;
        p1 = op1;
      } else {
        d2 = min(d2, od1);
      }
    }
    if ((KFKF ? d1 < TH_LOW : d1 <= TH_LOW) && (float)d1 < __fmul_rn(nnratio, (float)d2)) {
      if (lane == 0) {
        flag[p1] = 1;
        if (KFKF)
          M[ikf] = Fr.feats[so + q0 + p1];
        else
          M[Fr.feats[so + q0 + p1]] = ikf;
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  }
}

__device__ __forceinline__ int rot_bin(float a_kf, float a_f) {
  const float factor = 1.0f / HISTO_LENGTH;
  float rot = __fsub_rn(a_kf, a_f);
  if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
  int bin = (int)roundf(__fmul_rn(rot, factor));
  if (bin == HISTO_LENGTH) bin = 0;
  return bin;
}

// the rotation check of both searches: KFKF = false iterates the frame's matches (rot = angle(kf) -
// angle(frame), the histogram of frame indices), KFKF = true KF1's (rot = angle1 - angle2, histogram of
// idx1); n = the indexed side's feature counts
template <bool KFKF>
__global__ __launch_bounds__(256) void k_bow_rot(int cap, const int* __restrict__ n_idx,
                                                 const eao_keypoint_dev* __restrict__ kkps,
                                                 const eao_keypoint_dev* __restrict__ fkps, int check_ori,
                                                 int* __restrict__ f_match, int* __restrict__ nmatches,
                                                 const int* __restrict__ err) {
  __shared__ int hist[HISTO_LENGTH];
  __shared__ int keep[HISTO_LENGTH];
  __shared__ int s_cnt;
  const int s = blockIdx.x, t = threadIdx.x;
  const size_t so = (size_t)s * cap;
  const int n = min(n_idx[s], cap);
  if (err[s]) {  // a vocabulary node held more frame features than the search supports
    if (t == 0) nmatches[s] = EAO_E_CAPACITY;
    return;
  }
  if (t < HISTO_LENGTH) hist[t] = 0;
  if (t == 0) s_cnt = 0;
  __syncthreads();
  int* M = f_match + so;
  if (check_ori) {
    for (int i = t; i < n; i += 256) {
      const int k = M[i];
      if (k >= 0)
        atomicAdd(&hist[KFKF ? rot_bin(kkps[so + i].angle, fkps[so + k].angle)
                             : rot_bin(kkps[so + k].angle, fkps[so + i].angle)], 1);
    }
    __syncthreads();
    if (t == 0) {  // ComputeThreeMaxima (ORBmatcher.cc:1601-1642)
      int max1 = 0, max2 = 0, max3 = 0, i1 = -1, i2 = -1, i3 = -1;
      for (int i = 0; i < HISTO_LENGTH; i++) {
        const int v = hist[i];
        if (v > max1) {
          max3 = max2; max2 = max1; max1 = v;
          i3 = i2; i2 = i1; i1 = i;
        } else if (v > max2) {
          max3 = max2; max2 = v;
          i3 = i2; i2 = i;
        } else if (v > max3) {
          max3 = v;
          i3 = i;
        }
      }
      if (max2 < __fmul_rn(0.1f, (float)max1)) {
        i2 = -1;
        i3 = -1;
      } else if (max3 < __fmul_rn(0.1f, (float)max1)) {
        i3 = -1;
      }
      for (int i = 0; i < HISTO_LENGTH; i++) keep[i] = i == i1 || i == i2 || i == i3;
    }
    __syncthreads();
  }
  int c = 0;
  for (int i = t; i < n; i += 256) {
    const int k = M[i];
    if (k < 0) continue;
    if (check_ori && !keep[KFKF ? rot_bin(kkps[so + i].angle, fkps[so + k].angle)
                                : rot_bin(kkps[so + k].angle, fkps[so + i].angle)])
      M[i] = -1;
    else c++;
  }
  atomicAdd(&s_cnt, c);
  __syncthreads();
  if (t == 0) nmatches[s] = s_cnt;
}

}  // namespace

struct VocabEngine {
  int dev = 0, max_kps = 0, max_batch = 0, n_nodes = 0, L = 0, empty = 1;
  hipStream_t stream = nullptr;
  uint8_t* d_vdesc = nullptr;
  int* d_cstart = nullptr;
  int* d_cids = nullptr;
  int* d_word = nullptr;
  double* d_weight = nullptr;
  // per-feature scratch [max_batch][max_kps]
  int* d_fword = nullptr;
  double* d_fweight = nullptr;
  int* d_fnode = nullptr;
  // single-call staging: two sides of a search / one frame of a transform
  eao_keypoint_dev* d_kps = nullptr;  // [2][max_kps]
  uint8_t* d_desc = nullptr;          // [2][max_kps][32]
  uint8_t* d_valid = nullptr;         // [2][max_kps]
  int* d_i = nullptr;                 // [2][3 * max_kps + 1] node ids | start | feats, + counts
  double* d_ww = nullptr;             // [max_kps]
  int* d_out = nullptr;               // [max_kps + 16]
  int* d_err = nullptr;
  int* h_small = nullptr;             // pinned scalars of the single-frame calls
  std::vector<void*> ptrs;
  ~VocabEngine() {
    for (void* p : ptrs) (void)hipFree(p);
    if (h_small) (void)hipHostFree(h_small);
    if (stream) (void)hipStreamDestroy(stream);
  }
  template <typename Tp>
  hipError_t alloc(Tp** p, size_t bytes) {
    hipError_t r = hipMalloc((void**)p, bytes ? bytes : 16);
    if (r == hipSuccess) ptrs.push_back(*p);
    return r;
  }
  VocabDev view() const { return VocabDev{d_vdesc, d_cstart, d_cids, d_word, d_weight, L, empty}; }
};

}  // namespace eao

using namespace eao;

struct eao_vocab {
  VocabEngine e;
};

extern "C" {

int eao_vocab_create(int device, int n_nodes, const uint8_t* node_desc, const int32_t* parent,
                     const int32_t* word_id, const double* weight, int L, int max_kps, int max_batch,
                     eao_vocab** out) {
  if (!out) return EAO_E_ARG;
  *out = nullptr;
  if (!eao_device_ok(device)) {
    set_error("no usable gfx950 device (the engine has no CPU fallback)");
    return EAO_E_NODEVICE;
  }
  if (n_nodes < 0 || (n_nodes > 0 && (!node_desc || !parent || !word_id || !weight)) || L < 0 || max_kps < 1 ||
      max_kps > BOW_MAXN || max_batch < 1) {
    set_error("eao_vocab_create: bad arguments (max_kps in [1, 4096], vocabulary arrays)");
    return EAO_E_ARG;
  }
  for (int i = 1; i < n_nodes; i++)
    if (parent[i] < 0 || parent[i] >= i) {
      set_error("eao_vocab_create: parent[i] must lie in [0, i) (loadFromTextFile order)");
      return EAO_E_ARG;
    }
  eao_vocab* v = new eao_vocab();
  VocabEngine& e = v->e;
  e.dev = device;
  e.max_kps = max_kps;
  e.max_batch = max_batch;
  e.n_nodes = n_nodes;
  e.L = L;
  // children CSR in id order (loadFromTextFile pushes each child to its parent in file order)
  std::vector<int> cstart(n_nodes + 2, 0), cids(n_nodes > 0 ? n_nodes - 1 : 0);
  for (int i = 1; i < n_nodes; i++) cstart[parent[i] + 1]++;
  for (int i = 0; i < n_nodes; i++) cstart[i + 1] += cstart[i];
  {
    std::vector<int> fill(cstart.begin(), cstart.begin() + n_nodes);
    for (int i = 1; i < n_nodes; i++) cids[fill[parent[i]]++] = i;
  }
  bool any_word = false;
  for (int i = 0; i < n_nodes; i++) any_word |= word_id[i] >= 0;
  e.empty = !(any_word && n_nodes > 1 && cstart[1] > cstart[0]) ? 1 : 0;
  auto fail = [&](hipError_t r) {
    set_error(std::string("eao_vocab_create: ") + hipGetErrorString(r));
    delete v;
    return EAO_E_HIP;
  };
  hipError_t r;
  const size_t K = (size_t)max_kps, B = (size_t)max_batch;
  if ((r = hipSetDevice(device)) != hipSuccess) return fail(r);
  if ((r = hipStreamCreateWithFlags(&e.stream, hipStreamNonBlocking)) != hipSuccess) return fail(r);
  if ((r = e.alloc(&e.d_vdesc, 32 * (size_t)n_nodes)) != hipSuccess) return fail(r);
  if ((r = e.alloc(&e.d_cstart, sizeof(int) * (n_nodes + 1))) != hipSuccess) return fail(r);
  if ((r = e.alloc(&e.d_cids, sizeof(int) * cids.size())) != hipSuccess) return fail(r);
  if ((r = e.alloc(&e.d_word, sizeof(int) * n_nodes)) != hipSuccess) return fail(r);
  if ((r = e.alloc(&e.d_weight, sizeof(double) * n_nodes)) != hipSuccess) return fail(r);
  if ((r = e.alloc(&e.d_fword, sizeof(int) * K * B)) != hipSuccess) return fail(r);
  if ((r = e.alloc(&e.d_fweight, sizeof(double) * K * B)) != hipSuccess) return fail(r);
  if ((r = e.alloc(&e.d_fnode, sizeof(int) * K * B)) != hipSuccess) return fail(r);
  if ((r = e.alloc(&e.d_kps, sizeof(eao_keypoint_dev) * 2 * K)) != hipSuccess) return fail(r);
  if ((r = e.alloc(&e.d_desc, 64 * K)) != hipSuccess) return fail(r);
  if ((r = e.alloc(&e.d_valid, 2 * K)) != hipSuccess) return fail(r);
  if ((r = e.alloc(&e.d_i, sizeof(int) * 2 * (3 * K + 8))) != hipSuccess) return fail(r);
  if ((r = e.alloc(&e.d_ww, sizeof(double) * K)) != hipSuccess) return fail(r);
  if ((r = e.alloc(&e.d_out, sizeof(int) * (K + 16))) != hipSuccess) return fail(r);
  if ((r = e.alloc(&e.d_err, sizeof(int) * B)) != hipSuccess) return fail(r);
  if ((r = hipHostMalloc((void**)&e.h_small, sizeof(int) * 16, 0)) != hipSuccess) return fail(r);
  if (n_nodes > 0) {
    if ((r = hipMemcpy(e.d_vdesc, node_desc, 32 * (size_t)n_nodes, hipMemcpyHostToDevice)) != hipSuccess) return fail(r);
    if ((r = hipMemcpy(e.d_cstart, cstart.data(), sizeof(int) * (n_nodes + 1), hipMemcpyHostToDevice)) != hipSuccess)
      return fail(r);
    if (!cids.empty() &&
        (r = hipMemcpy(e.d_cids, cids.data(), sizeof(int) * cids.size(), hipMemcpyHostToDevice)) != hipSuccess)
      return fail(r);
    if ((r = hipMemcpy(e.d_word, word_id, sizeof(int) * n_nodes, hipMemcpyHostToDevice)) != hipSuccess) return fail(r);
    if ((r = hipMemcpy(e.d_weight, weight, sizeof(double) * n_nodes, hipMemcpyHostToDevice)) != hipSuccess)
      return fail(r);
  }
  *out = v;
  return EAO_OK;
}

int eao_vocab_destroy(eao_vocab* v) {
  delete v;
  return EAO_OK;
}

int eao_bow_transform_batch_device(eao_vocab* v, int nframes, int cap, const int32_t* d_counts,
                                   const uint8_t* d_desc, int levelsup, int32_t* d_word_ids,
                                   double* d_word_weights, int32_t* d_n_words, int32_t* d_node_ids,
                                   int32_t* d_node_start, int32_t* d_node_feats, int32_t* d_n_nodes,
                                   void* stream) {
  if (!v || nframes < 0 || nframes > v->e.max_batch || cap < 1 || cap > v->e.max_kps ||
      (nframes > 0 && (!d_counts || !d_desc || !d_word_ids || !d_word_weights || !d_n_words || !d_node_ids ||
                       !d_node_start || !d_node_feats || !d_n_nodes))) {
    set_error("eao_bow_transform_batch_device: bad arguments (nframes <= max_batch, cap <= max_kps)");
    return EAO_E_ARG;
  }
  if (nframes == 0) return EAO_OK;
  VocabEngine& e = v->e;
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  hipStream_t s = stream ? (hipStream_t)stream : e.stream;
  hipLaunchKernelGGL(k_bow_words, dim3((cap + 255) / 256, nframes), dim3(256), 0, s, e.view(), cap, d_counts, d_desc,
                     levelsup, e.d_fword, e.d_fweight, e.d_fnode);
  hipLaunchKernelGGL(k_bow_build, dim3(nframes), dim3(1024), 0, s, cap, d_counts, e.d_fword, e.d_fweight, e.d_fnode,
                     d_word_ids, d_word_weights, d_n_words, d_node_ids, d_node_start, d_node_feats, d_n_nodes);
  EAO_HIP_CHECK(hipGetLastError());
  return EAO_OK;
}

int eao_bow_transform(eao_vocab* v, int n, const uint8_t* desc, int levelsup, int32_t* word_ids,
                      double* word_weights, int32_t* n_words, int32_t* node_ids, int32_t* node_start,
                      int32_t* node_feats, int32_t* n_nodes) {
  if (!v || n < 0 || n > v->e.max_kps || (n > 0 && !desc) || !word_ids || !word_weights || !n_words ||
      !node_ids || !node_start || !node_feats || !n_nodes) {
    set_error("eao_bow_transform: bad arguments (n outside [0, max_kps] or null buffer)");
    return EAO_E_ARG;
  }
  VocabEngine& e = v->e;
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  hipStream_t s = e.stream;
  const int K = e.max_kps, cap = K;
  int* d_cnt = e.d_i + 6 * K + 8;  // counts / outputs: [0] n, [1] n_words, [2] n_nodes
  int* d_ids = e.d_i;
  int* d_start = e.d_i + K;
  int* d_feats = e.d_i + 2 * K + 1;
  int* d_wid = e.d_out;
  e.h_small[0] = n;
  EAO_HIP_CHECK(hipMemcpyAsync(d_cnt, e.h_small, sizeof(int), hipMemcpyHostToDevice, s));
  if (n > 0) EAO_HIP_CHECK(hipMemcpyAsync(e.d_desc, desc, 32 * (size_t)n, hipMemcpyHostToDevice, s));
  int rc = eao_bow_transform_batch_device(v, 1, cap, d_cnt, e.d_desc, levelsup, d_wid, e.d_ww, d_cnt + 1, d_ids,
                                          d_start, d_feats, d_cnt + 2, s);
  if (rc) return rc;
  EAO_HIP_CHECK(hipMemcpyAsync(e.h_small + 4, d_cnt, 3 * sizeof(int), hipMemcpyDeviceToHost, s));
  EAO_HIP_CHECK(hipStreamSynchronize(s));
  const int hc[3] = {e.h_small[4], e.h_small[5], e.h_small[6]};
  *n_words = hc[1];
  *n_nodes = hc[2];
  if (hc[1] > 0) {
    EAO_HIP_CHECK(hipMemcpy(word_ids, d_wid, sizeof(int) * hc[1], hipMemcpyDeviceToHost));
    EAO_HIP_CHECK(hipMemcpy(word_weights, e.d_ww, sizeof(double) * hc[1], hipMemcpyDeviceToHost));
  }
  EAO_HIP_CHECK(hipMemcpy(node_start, d_start, sizeof(int) * (hc[2] + 1), hipMemcpyDeviceToHost));
  if (hc[2] > 0) {
    EAO_HIP_CHECK(hipMemcpy(node_ids, d_ids, sizeof(int) * hc[2], hipMemcpyDeviceToHost));
    if (node_start[hc[2]] > 0)
      EAO_HIP_CHECK(hipMemcpy(node_feats, d_feats, sizeof(int) * node_start[hc[2]], hipMemcpyDeviceToHost));
  }
  return EAO_OK;
}

int eao_search_by_bow_batch_device(eao_vocab* v, float nnratio, int check_ori, int nsearch, int cap,
                                   const eao_keypoint* d_kf_kps, const uint8_t* d_kf_desc,
                                   const uint8_t* d_kf_mp_valid, const int32_t* d_kf_nn,
                                   const int32_t* d_kf_node_ids, const int32_t* d_kf_node_start,
                                   const int32_t* d_kf_node_feats, const int32_t* d_n_f,
                                   const eao_keypoint* d_f_kps, const uint8_t* d_f_desc,
                                   const int32_t* d_f_nn, const int32_t* d_f_node_ids,
                                   const int32_t* d_f_node_start, const int32_t* d_f_node_feats,
                                   int32_t* d_f_match, int32_t* d_nmatches, void* stream) {
  if (!v || nsearch < 0 || nsearch > v->e.max_batch || cap < 1 || cap > v->e.max_kps) {
    set_error("eao_search_by_bow_batch_device: bad arguments (nsearch <= max_batch, cap in [1, max_kps])");
    return EAO_E_ARG;
  }
  if (nsearch == 0) return EAO_OK;
  VocabEngine& e = v->e;
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  hipStream_t s = stream ? (hipStream_t)stream : e.stream;
  const SearchSlot K{(const eao_keypoint_dev*)d_kf_kps, d_kf_desc, d_kf_mp_valid, d_kf_nn, d_kf_node_ids,
                     d_kf_node_start, d_kf_node_feats};
  const SearchSlot F{(const eao_keypoint_dev*)d_f_kps, d_f_desc, nullptr, d_f_nn, d_f_node_ids, d_f_node_start,
                     d_f_node_feats};
  EAO_HIP_CHECK(hipMemsetAsync(d_f_match, 0xff, sizeof(int) * (size_t)nsearch * cap, s));
  EAO_HIP_CHECK(hipMemsetAsync(e.d_err, 0, sizeof(int) * nsearch, s));
  hipLaunchKernelGGL(k_bow_search<false>, dim3((cap + 3) / 4, nsearch), dim3(256), 0, s, cap, K, F, nnratio,
                     d_f_match, e.d_err);
  hipLaunchKernelGGL(k_bow_rot<false>, dim3(nsearch), dim3(256), 0, s, cap, d_n_f, K.kps, F.kps, check_ori,
                     d_f_match, d_nmatches, e.d_err);
  EAO_HIP_CHECK(hipGetLastError());
  return EAO_OK;
}

int eao_search_by_bow_kf_batch_device(eao_vocab* v, float nnratio, int check_ori, int nsearch, int cap,
                                      const int32_t* d_n1, const eao_keypoint* d_kps1, const uint8_t* d_desc1,
                                      const uint8_t* d_valid1, const int32_t* d_nn1, const int32_t* d_node_ids1,
                                      const int32_t* d_node_start1, const int32_t* d_node_feats1,
                                      const eao_keypoint* d_kps2, const uint8_t* d_desc2, const uint8_t* d_valid2,
                                      const int32_t* d_nn2, const int32_t* d_node_ids2,
                                      const int32_t* d_node_start2, const int32_t* d_node_feats2,
                                      int32_t* d_match12, int32_t* d_nmatches, void* stream) {
  if (!v || nsearch < 0 || nsearch > v->e.max_batch || cap < 1 || cap > v->e.max_kps) {
    set_error("eao_search_by_bow_kf_batch_device: bad arguments (nsearch <= max_batch, cap in [1, max_kps])");
    return EAO_E_ARG;
  }
  if (nsearch == 0) return EAO_OK;
  VocabEngine& e = v->e;
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  hipStream_t s = stream ? (hipStream_t)stream : e.stream;
  const SearchSlot K1{(const eao_keypoint_dev*)d_kps1, d_desc1, d_valid1, d_nn1, d_node_ids1, d_node_start1,
                      d_node_feats1};
  const SearchSlot K2{(const eao_keypoint_dev*)d_kps2, d_desc2, d_valid2, d_nn2, d_node_ids2, d_node_start2,
                      d_node_feats2};
  EAO_HIP_CHECK(hipMemsetAsync(d_match12, 0xff, sizeof(int) * (size_t)nsearch * cap, s));
  EAO_HIP_CHECK(hipMemsetAsync(e.d_err, 0, sizeof(int) * nsearch, s));
  hipLaunchKernelGGL(k_bow_search<true>, dim3((cap + 3) / 4, nsearch), dim3(256), 0, s, cap, K1, K2, nnratio,
                     d_match12, e.d_err);
  hipLaunchKernelGGL(k_bow_rot<true>, dim3(nsearch), dim3(256), 0, s, cap, d_n1, K1.kps, K2.kps, check_ori,
                     d_match12, d_nmatches, e.d_err);
  EAO_HIP_CHECK(hipGetLastError());
  return EAO_OK;
}

// one search of either kind on host buffers: side 1 (keyframe / KF1) and side 2 (frame / KF2)
// staged into the handle's two slots, the batched path on one search, the result back
static int search_single(eao_vocab* v, bool kfkf, const char* name, float nnratio, int check_ori, int n1,
                         const eao_keypoint* kps1, const uint8_t* desc1, const uint8_t* valid1, int nn1,
                         const int32_t* ids1, const int32_t* st1, const int32_t* ft1, int n2,
                         const eao_keypoint* kps2, const uint8_t* desc2, const uint8_t* valid2, int nn2,
                         const int32_t* ids2, const int32_t* st2, const int32_t* ft2, int32_t* out) {
  if (!v || n1 < 0 || n2 < 0 || n1 > v->e.max_kps || n2 > v->e.max_kps || nn1 < 0 || nn2 < 0 || nn1 > n1 ||
      nn2 > n2 || !out || (n1 > 0 && (!kps1 || !desc1 || !valid1)) ||
      (n2 > 0 && (!kps2 || !desc2 || (kfkf && !valid2))) || (nn1 > 0 && (!ids1 || !st1 || !ft1)) ||
      (nn2 > 0 && (!ids2 || !st2 || !ft2))) {
    set_error(std::string(name) + ": bad arguments (sizes outside [0, max_kps] or null buffer)");
    return EAO_E_ARG;
  }
  const int n_out = kfkf ? n1 : n2;  // the side the result is indexed by
  if (n_out == 0) return 0;
  VocabEngine& e = v->e;
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  hipStream_t s = e.stream;
  const int K = e.max_kps;
  // staging: side 1 and side 2; the node CSR of side k at d_i + k * (3K + 8), then its node and
  // feature counts
  int* I1 = e.d_i;
  int* I2 = e.d_i + 3 * K + 8;
  const int nf1 = nn1 > 0 ? st1[nn1] : 0, nf2 = nn2 > 0 ? st2[nn2] : 0;
  if (nf1 > n1 || nf2 > n2) {
    set_error(std::string(name) + ": a FeatureVector lists more features than the side has");
    return EAO_E_ARG;
  }
  // the kernel indexes descriptors / flags / matches with these values and binary-searches the
  // node ids: every feature index in range, node starts non-decreasing, node ids ascending
  auto fv_ok = [](int nn, const int32_t* ids, const int32_t* st, const int32_t* ft, int nfeat) {
    if (nn > 0 && st[0] != 0) return false;
    for (int i = 0; i < nn; i++)
      if (st[i + 1] < st[i] || (i > 0 && ids[i] <= ids[i - 1])) return false;
    const int tot = nn > 0 ? st[nn] : 0;
    for (int k = 0; k < tot; k++)
      if (ft[k] < 0 || ft[k] >= nfeat) return false;
    return true;
  };
  if (!fv_ok(nn1, ids1, st1, ft1, n1) || !fv_ok(nn2, ids2, st2, ft2, n2)) {
    set_error(std::string(name) + ": malformed FeatureVector (feature index out of range, node starts "
              "decreasing or node ids not ascending)");
    return EAO_E_ARG;
  }
  if (n1 > 0) {
    EAO_HIP_CHECK(hipMemcpyAsync(e.d_kps, kps1, sizeof(eao_keypoint) * n1, hipMemcpyHostToDevice, s));
    EAO_HIP_CHECK(hipMemcpyAsync(e.d_desc, desc1, 32 * (size_t)n1, hipMemcpyHostToDevice, s));
    EAO_HIP_CHECK(hipMemcpyAsync(e.d_valid, valid1, n1, hipMemcpyHostToDevice, s));
  }
  if (n2 > 0) {
    EAO_HIP_CHECK(hipMemcpyAsync(e.d_kps + K, kps2, sizeof(eao_keypoint) * n2, hipMemcpyHostToDevice, s));
    EAO_HIP_CHECK(hipMemcpyAsync(e.d_desc + 32 * (size_t)K, desc2, 32 * (size_t)n2, hipMemcpyHostToDevice, s));
    if (kfkf) EAO_HIP_CHECK(hipMemcpyAsync(e.d_valid + K, valid2, n2, hipMemcpyHostToDevice, s));
  }
  auto up_fv = [&](int* base, int nn, const int32_t* ids, const int32_t* st, const int32_t* ft, int nf, int n,
                   int* hslot) -> int {
    hslot[0] = nn;
    hslot[1] = n;
    EAO_HIP_CHECK(hipMemcpyAsync(base + 3 * K + 4, hslot, 2 * sizeof(int), hipMemcpyHostToDevice, s));
    if (nn > 0) {
      EAO_HIP_CHECK(hipMemcpyAsync(base, ids, sizeof(int) * nn, hipMemcpyHostToDevice, s));
      EAO_HIP_CHECK(hipMemcpyAsync(base + K, st, sizeof(int) * (nn + 1), hipMemcpyHostToDevice, s));
      if (nf > 0) EAO_HIP_CHECK(hipMemcpyAsync(base + 2 * K + 1, ft, sizeof(int) * nf, hipMemcpyHostToDevice, s));
    }
    return EAO_OK;
  };
  int rc = up_fv(I1, nn1, ids1, st1, ft1, nf1, n1, e.h_small);
  if (!rc) rc = up_fv(I2, nn2, ids2, st2, ft2, nf2, n2, e.h_small + 2);
  if (rc) return rc;
  const eao_keypoint* k1 = (const eao_keypoint*)e.d_kps;
  const eao_keypoint* k2 = (const eao_keypoint*)(e.d_kps + K);
  if (kfkf)
    rc = eao_search_by_bow_kf_batch_device(v, nnratio, check_ori, 1, K, I1 + 3 * K + 5, k1, e.d_desc, e.d_valid,
                                           I1 + 3 * K + 4, I1, I1 + K, I1 + 2 * K + 1, k2, e.d_desc + 32 * (size_t)K,
                                           e.d_valid + K, I2 + 3 * K + 4, I2, I2 + K, I2 + 2 * K + 1, e.d_out,
                                           e.d_out + K, s);
  else
    rc = eao_search_by_bow_batch_device(v, nnratio, check_ori, 1, K, k1, e.d_desc, e.d_valid, I1 + 3 * K + 4, I1,
                                        I1 + K, I1 + 2 * K + 1, I2 + 3 * K + 5, k2, e.d_desc + 32 * (size_t)K,
                                        I2 + 3 * K + 4, I2, I2 + K, I2 + 2 * K + 1, e.d_out, e.d_out + K, s);
  if (rc) return rc;
  EAO_HIP_CHECK(hipMemcpyAsync(out, e.d_out, sizeof(int) * n_out, hipMemcpyDeviceToHost, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.h_small + 4, e.d_out + K, sizeof(int), hipMemcpyDeviceToHost, s));
  EAO_HIP_CHECK(hipStreamSynchronize(s));
  const int nm = e.h_small[4];
  if (nm < 0) {
    set_error(std::string(name) + ": a vocabulary node holds more than 1024 features of the second side");
    return EAO_E_CAPACITY;
  }
  return nm;
}

int eao_search_by_bow(eao_vocab* v, float nnratio, int check_ori, int n_kf, const eao_keypoint* kf_kps,
                      const uint8_t* kf_desc, const uint8_t* kf_mp_valid, int kf_nn,
                      const int32_t* kf_node_ids, const int32_t* kf_node_start,
                      const int32_t* kf_node_feats, int n_f, const eao_keypoint* f_kps,
                      const uint8_t* f_desc, int f_nn, const int32_t* f_node_ids,
                      const int32_t* f_node_start, const int32_t* f_node_feats, int32_t* f_match) {
  return search_single(v, false, "eao_search_by_bow", nnratio, check_ori, n_kf, kf_kps, kf_desc, kf_mp_valid, kf_nn,
                       kf_node_ids, kf_node_start, kf_node_feats, n_f, f_kps, f_desc, nullptr, f_nn, f_node_ids,
                       f_node_start, f_node_feats, f_match);
}

int eao_search_by_bow_kf(eao_vocab* v, float nnratio, int check_ori, int n1, const eao_keypoint* kps1,
                         const uint8_t* desc1, const uint8_t* valid1, int nn1, const int32_t* node_ids1,
                         const int32_t* node_start1, const int32_t* node_feats1, int n2, const eao_keypoint* kps2,
                         const uint8_t* desc2, const uint8_t* valid2, int nn2, const int32_t* node_ids2,
                         const int32_t* node_start2, const int32_t* node_feats2, int32_t* match12) {
  return search_single(v, true, "eao_search_by_bow_kf", nnratio, check_ori, n1, kps1, desc1, valid1, nn1, node_ids1,
                       node_start1, node_feats1, n2, kps2, desc2, valid2, nn2, node_ids2, node_start2, node_feats2,
                       match12);
}

}  // extern "C"
