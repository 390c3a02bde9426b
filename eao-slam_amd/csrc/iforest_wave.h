// iforest_wave.h -- one-wave building blocks of the isolation-forest kernel
// (assoc.hip): the libstdc++ mt19937 / Lemire / canonical-float draw stream
// of a wave, order-preserving float keys, wave min/max and a 3-way 64-lane
// bitonic sort. Included by assoc.hip and the tools/micro benchmarks.
#pragma once
#include <climits>
#include "common.h"

namespace eao {

// Compiler barrier between the phases of a one-wave algorithm: a wave's LDS
// operations execute in program order, so only compiler reordering across
// lanes' data dependencies has to be prevented.
#define WAVE_FENCE() __asm__ volatile("" ::: "memory")

// std::mt19937 for one wave: state in LDS, tempered outputs buffered one per
// lane in a VGPR and handed out in stream order with v_readlane.
struct WaveRng {
  uint32_t* mt;  // LDS [624]
  int idx;       // next untempered state word (uniform)
  int tw;        // twists since the state the generator started from (draw count = 624 tw + idx - unread)
  uint32_t buf;  // lane j: draw number (base + j) of the current chunk
  uint32_t bufd;  // the same draw as uniform_int<uint32>(0, 2) (Lemire), 3 = rejected
  float buff;     // the same draw as generate_canonical<float, 24>
  int bp, blen;   // uniform read position / valid length of buf

  __device__ void seed(uint32_t s) {
    if (lane_id() == 0) {
      uint32_t x = s;
      mt[0] = x;
      for (int i = 1; i < 624; i++) {
        x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)i;
        mt[i] = x;
      }
    }
    idx = 624;
    tw = -1;
    bp = blen = 0;
    WAVE_FENCE();
  }
  // libstdc++ _M_gen_rand in chunks of 64 words in increasing order: word k
  // reads k+1 (old) and (k+397)%624 (new for k >= 227, written by an earlier
  // chunk), exactly the in-place order of the sequential recurrence.
  __device__ void twist() {
    const int l = lane_id();
    for (int c0 = 0; c0 < 623; c0 += 64) {
      const int k = c0 + l;
      uint32_t nv = 0;
      if (k < 623) {
        const uint32_t y = (mt[k] & 0x80000000u) | (mt[k + 1] & 0x7fffffffu);
        nv = mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      }
      WAVE_FENCE();
      if (k < 623) mt[k] = nv;
      WAVE_FENCE();
    }
    if (l == 0) {
      const uint32_t y = (mt[623] & 0x80000000u) | (mt[0] & 0x7fffffffu);
      mt[623] = mt[396] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    WAVE_FENCE();
    idx = 0;
    tw++;
  }
  __device__ void refill() {
    idx = __builtin_amdgcn_readfirstlane(idx);  // uniform state: keep it scalar
    if (idx >= 624) twist();
    blen = __builtin_amdgcn_readfirstlane(min(64, 624 - idx));
    const int l = lane_id();
    uint32_t y = l < blen ? mt[idx + l] : 0u;
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    buf = y;
    // both interpretations of every draw, precomputed off the build's critical chain:
    // Lemire over range 3 rejects low = y * 3 < 1, i.e. y == 0
    bufd = y == 0u ? 3u : __umulhi(y, 3u);
    float r = fmul((float)y, 0x1p-32f);               // == y / 2^32 exactly (power-of-two scale)
    buff = r >= 1.0f ? __uint_as_float(0x3f7fffffu) : r;  // nextafter(1, 0)
    idx = __builtin_amdgcn_readfirstlane(idx + blen);
    bp = 0;
  }
  __device__ uint32_t next() {
    if (bp >= blen) refill();
    return (uint32_t)__builtin_amdgcn_readlane((int)buf, bp++);
  }
  // uniform_int_distribution<uint32_t>(0, range-1) with a 32-bit URNG (Lemire)
  __device__ uint32_t lemire(uint32_t range) {
    uint64_t product = (uint64_t)next() * (uint64_t)range;
    uint32_t low = (uint32_t)product;
    if (low < range) {
      const uint32_t threshold = (uint32_t)(0u - range) % range;
      while (low < threshold) {
        product = (uint64_t)next() * (uint64_t)range;
        low = (uint32_t)product;
      }
    }
    return (uint32_t)(product >> 32);
  }
  // uniform_int_distribution<uint32_t>(0, 2): lemire(3) from the precomputed lane values
  __device__ uint32_t dim3() {
    uint32_t d;
    do {
      // the read position is wave-uniform: readfirstlane keeps it (and the refill test) scalar
      bp = __builtin_amdgcn_readfirstlane(bp);
      blen = __builtin_amdgcn_readfirstlane(blen);
      if (bp >= blen) refill();
      d = (uint32_t)__builtin_amdgcn_readlane((int)bufd, bp++);
    } while (d == 3u);
    return d;
  }
  // uniform_real_distribution<float>(a, b): generate_canonical<float, 24>
  __device__ float uniform_real(float a, float b) {
    bp = __builtin_amdgcn_readfirstlane(bp);
    blen = __builtin_amdgcn_readfirstlane(blen);
    if (bp >= blen) refill();
    const float ret = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(buff), bp++));
    return fadd(fmul(ret, fsub(b, a)), a);
  }
};

__device__ __forceinline__ double iforest_c(uint32_t n) {  // CalculateC, isolation_forest.h:97-118
  if (n > 2) {
    const double h = log((double)(n - 1)) + 0.5772156649;
    return __dsub_rn(2.0 * h, (2.0 * (double)(n - 1)) / (double)n);
  } else if (n == 2)
    return 1.0;
  return 0.0;
}

// order-preserving int key of a finite float (-0 folded onto +0, so key
// order and equality are exactly the float comparisons); kfloat inverts it
__device__ __forceinline__ int fkey(float f) {
  int b = __float_as_int(f);
  b = b == (int)0x80000000 ? 0 : b;
  return b ^ ((b >> 31) & 0x7fffffff);
}
__device__ __forceinline__ float kfloat(int k) { return __int_as_float(k ^ ((k >> 31) & 0x7fffffff)); }

// wave-wide min and max of int keys, uniform results: DPP-fused min/max
// within rows, then permlane16/32 swaps across rows (gfx950)
__device__ __forceinline__ void wave_minmax_key(int& mn, int& mx) {
  mn = min(mn, __builtin_amdgcn_update_dpp(0, mn, 0xB1, 0xF, 0xF, false));  // quad_perm [1,0,3,2]
  mx = max(mx, __builtin_amdgcn_update_dpp(0, mx, 0xB1, 0xF, 0xF, false));
  mn = min(mn, __builtin_amdgcn_update_dpp(0, mn, 0x4E, 0xF, 0xF, false));  // quad_perm [2,3,0,1]
  mx = max(mx, __builtin_amdgcn_update_dpp(0, mx, 0x4E, 0xF, 0xF, false));
  mn = min(mn, __builtin_amdgcn_update_dpp(0, mn, 0x141, 0xF, 0xF, false));  // row_half_mirror
  mx = max(mx, __builtin_amdgcn_update_dpp(0, mx, 0x141, 0xF, 0xF, false));
  mn = min(mn, __builtin_amdgcn_update_dpp(0, mn, 0x140, 0xF, 0xF, false));  // row_mirror
  mx = max(mx, __builtin_amdgcn_update_dpp(0, mx, 0x140, 0xF, 0xF, false));
  auto a = __builtin_amdgcn_permlane16_swap(mn, mn, false, false);
  auto b = __builtin_amdgcn_permlane16_swap(mx, mx, false, false);
  mn = min((int)a[0], (int)a[1]);
  mx = max((int)b[0], (int)b[1]);
  a = __builtin_amdgcn_permlane32_swap(mn, mn, false, false);
  b = __builtin_amdgcn_permlane32_swap(mx, mx, false, false);
  mn = __builtin_amdgcn_readfirstlane(min((int)a[0], (int)a[1]));
  mx = __builtin_amdgcn_readfirstlane(max((int)b[0], (int)b[1]));
}

__host__ __device__ __forceinline__ size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

// tree node record in LDS: x = dim + 1 (bits 0-1) | right child id << 16 for a split,
// count << 2 for a leaf (count < 16384); y = the split's float bits. The right link is
// written later, into the upper half of x (a 16-bit store after the record's own store),
// so the score walk reads one record per level.
__device__ __forceinline__ void set_right(uint2* nodes, int id, int link) {
  ((uint16_t*)nodes)[4 * id + 1] = (uint16_t)link;
}

// lane l <- lane l ^ J (J a power of two < 64): DPP within quads, swizzle
// within 32, permlane swaps across rows / halves (gfx950)
template <int J>
__device__ __forceinline__ int xor_lane(int v) {
  if constexpr (J == 1) {
    return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  } else if constexpr (J == 2) {
    return __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
  } else if constexpr (J == 4 || J == 8) {
    return __builtin_amdgcn_ds_swizzle(v, 0x1f | (J << 10));  // bit mode: xor J within 32
  } else if constexpr (J == 16) {
    auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (lane_id() & 16) ? (int)a[0] : (int)a[1];
  } else {
    auto a = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (lane_id() & 32) ? (int)a[0] : (int)a[1];
  }
}
template <int J>
__device__ __forceinline__ uint64_t xor_lane64(uint64_t v) {
  const uint32_t lo = (uint32_t)xor_lane<J>((int)(uint32_t)v), hi = (uint32_t)xor_lane<J>((int)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
template <int K, int J>
__device__ __forceinline__ void bitonic_step3(uint64_t& a, uint64_t& b, uint64_t& c) {
  const int l = lane_id();
  const bool wantmin = ((l & J) == 0) == ((l & K) == 0);
  const uint64_t pa = xor_lane64<J>(a), pb = xor_lane64<J>(b), pc = xor_lane64<J>(c);
  a = wantmin ? (pa < a ? pa : a) : (pa > a ? pa : a);
  b = wantmin ? (pb < b ? pb : b) : (pb > b ? pb : b);
  c = wantmin ? (pc < c ? pc : c) : (pc > c ? pc : c);
}
template <int K, int J>
__device__ __forceinline__ void bitonic_merge3(uint64_t& a, uint64_t& b, uint64_t& c) {
  bitonic_step3<K, J>(a, b, c);
  if constexpr (J > 1) bitonic_merge3<K, J / 2>(a, b, c);
}
template <int K>
__device__ __forceinline__ void bitonic_sort3(uint64_t& a, uint64_t& b, uint64_t& c) {
  if constexpr (K > 2) bitonic_sort3<K / 2>(a, b, c);
  bitonic_merge3<K, K / 2>(a, b, c);
}
// v_writelane_b32: lane `l` (uniform) of v <- the uniform value x
extern "C" __device__ int eao_llvm_writelane(int x, int l, int old) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ void writelane(int& v, int x, int l) { v = eao_llvm_writelane(x, l, v); }
// ascending sort of three 64-lane sequences at once (lane = rank afterwards)
__device__ __forceinline__ void wave_sort3(uint64_t& a, uint64_t& b, uint64_t& c) { bitonic_sort3<64>(a, b, c); }

}  // namespace eao

namespace eao {

// Node::Build (isolation_forest.h:165-224) of a whole subtree of 2..64 items
// (one per lane, order-preserving int keys kx/ky/kz) by one wave, in rank
// space: the items are sorted once per dimension, a node is a 64-bit set of
// ranks per dimension, so a node's min / max are its lowest / highest set
// rank (scalar bit scans + two readlanes) and the split's left side is a
// prefix of the rank order; the children's rank sets in all three dimensions
// come from one ballot each through the item permutation. Draws are taken
// from g exactly as the sequential build takes them (dim: Lemire over 3,
// split: uniform_real(min, max)); leaves (by count or depth) consume none and
// are recorded without a loop trip. Node records (x = dim + 1 | right child id << 16 for
// a split, count << 2 for a leaf; y = split bits) go to nodes for ids [me, nn), preorder;
// a right link is a 16-bit store into the upper half of x once the right child has its id;
// the caller has allocated `me` (nn == me + 1) and checked 2 <= cnt,
// depth < maxDepth. Returns 1 when Node::Build fails (empty right range).
// per dimension: the sorted key at rank (lane), the item at rank (lane), the rank of item (lane)
struct RankTab {
  int sx, sy, sz, px, py, pz, rx, ry, rz;
};
// LDS image of a RankTab (the forest kernel's helper waves prepare subtrees ahead of wave 0)
struct RankSlot {
  int s[3][64];
  uint8_t p[3][64], r[3][64];
};
__device__ __forceinline__ void rank_store(RankSlot* S, const RankTab& t) {
  const int l = lane_id();
  S->s[0][l] = t.sx;
  S->s[1][l] = t.sy;
  S->s[2][l] = t.sz;
  S->p[0][l] = (uint8_t)t.px;
  S->p[1][l] = (uint8_t)t.py;
  S->p[2][l] = (uint8_t)t.pz;
  S->r[0][l] = (uint8_t)t.rx;
  S->r[1][l] = (uint8_t)t.ry;
  S->r[2][l] = (uint8_t)t.rz;
}
__device__ __forceinline__ RankTab rank_load(const RankSlot* S) {
  const int l = lane_id();
  RankTab t;
  t.sx = S->s[0][l];
  t.sy = S->s[1][l];
  t.sz = S->s[2][l];
  t.px = S->p[0][l];
  t.py = S->p[1][l];
  t.pz = S->p[2][l];
  t.rx = S->r[0][l];
  t.ry = S->r[1][l];
  t.rz = S->r[2][l];
  return t;
}

// the subtree's items sorted once per dimension (rank_subtree's preparation; it depends on the
// items only, not on the draw stream)
__device__ __forceinline__ RankTab rank_prep(int kx, int ky, int kz, int cnt) {
  const int lane = lane_id();
  auto sk64 = [&](int k) { return ((uint64_t)((uint32_t)k ^ 0x80000000u) << 32) | (uint32_t)lane; };
  uint64_t vx = sk64(lane < cnt ? kx : INT_MAX), vy = sk64(lane < cnt ? ky : INT_MAX),
           vz = sk64(lane < cnt ? kz : INT_MAX);
  // the items sit in lanes [0, cnt): a bitonic network over the next power of two >= cnt
  // lanes sorts them (lanes beyond hold INT_MAX keys whatever order they end in, and no
  // node ever contains them); 6 / 10 / 15 steps instead of 21 for cnt <= 8 / 16 / 32
  if (cnt > 32)
    wave_sort3(vx, vy, vz);
  else if (cnt > 16)
    bitonic_sort3<32>(vx, vy, vz);
  else if (cnt > 8)
    bitonic_sort3<16>(vx, vy, vz);
  else
    bitonic_sort3<8>(vx, vy, vz);
  // rank r (this lane): sorted key s*, item p*; item l (this lane): rank r*
  const int sx = (int)((uint32_t)(vx >> 32) ^ 0x80000000u), px = (int)(uint32_t)vx;
  const int sy = (int)((uint32_t)(vy >> 32) ^ 0x80000000u), py = (int)(uint32_t)vy;
  const int sz = (int)((uint32_t)(vz >> 32) ^ 0x80000000u), pz = (int)(uint32_t)vz;
  const int rx = __builtin_amdgcn_ds_permute(px << 2, lane);
  const int ry = __builtin_amdgcn_ds_permute(py << 2, lane);
  const int rz = __builtin_amdgcn_ds_permute(pz << 2, lane);
  return RankTab{sx, sy, sz, px, py, pz, rx, ry, rz};
}

__device__ __forceinline__ int rank_build(WaveRng& g, const RankTab& tb, int cnt, int depth, int maxDepth, int me,
                                          int& nn, uint2* nodes) {
  const int lane = lane_id();
  const int sx = tb.sx, sy = tb.sy, sz = tb.sz, px = tb.px, py = tb.py, pz = tb.pz, rx = tb.rx, ry = tb.ry,
            rz = tb.rz;
  // sorted values as floats (-0 folded): min / max / split compare in float
  const float fx = kfloat(sx), fy = kfloat(sy), fz = kfloat(sz);
  // a node is its set of items (bit l = item l); per node only the drawn dimension's
  // rank set is formed (one ballot through the item permutation) and the left
  // child's items come back through the inverse one
  uint64_t S = cnt == 64 ? ~0ull : ((1ull << cnt) - 1ull);
  int d = depth, node = me, cn = cnt, ssp = 0, bad = 0;
  // Node records and right links go straight to LDS from lane 0 (stores: off the chain).
  // The loop is written for few taken branches (each costs ~34 cycles on one wave):
  // both possible leaf-child records are stored unconditionally at ids nn and nn + 1 --
  // a record at an id that is not (yet) that node's is overwritten later in program
  // order, since every id up to the final nn gets exactly one real record after it
  // (the node array has room for the two look-ahead ids) -- and the stack push is an
  // unconditional writelane whose depth only advances when it is meant.
  auto put = [&](int id, uint32_t x, uint32_t y) {
    if (lane == 0) nodes[id] = make_uint2(x, y);
  };
  // pending right children, entry e in lane e: item set (q0, q1), depth | leaf flag
  // (bit 8), parent id
  int q0 = 0, q1 = 0, q2 = 0, q3 = 0;
  while (true) {
    // the current node (items S, count cn, depth d, id node) is not a leaf by count
    // or depth
    const uint32_t dim = g.dim3();
    const int pk = dim == 0 ? px : (dim == 1 ? py : pz);  // item at rank (lane)
    const int rk = dim == 0 ? rx : (dim == 1 ? ry : rz);  // rank of item (lane)
    const float fk = dim == 0 ? fx : (dim == 1 ? fy : fz);
    const uint64_t md = ballot((S >> pk) & 1ull);  // the node's ranks in this dimension
    const int lo = __builtin_ctzll(md), hi = 63 - __builtin_clzll(md);
    const float mn = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, fk), lo));
    const float mx = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, fk), hi));
    const bool eq = __builtin_bit_cast(int, mn) == __builtin_bit_cast(int, mx);
    // the split draw is read whatever the outcome and consumed only when min != max
    g.bp = __builtin_amdgcn_readfirstlane(g.bp);
    g.blen = __builtin_amdgcn_readfirstlane(g.blen);
    if (g.bp >= g.blen) g.refill();
    const float r = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(g.buff), g.bp));
    g.bp += eq ? 0 : 1;
    const float split = fadd(fmul(r, fsub(mx, mn)), mn);
    const uint64_t lm = md & ballot(fk < split);  // ranks below the split: a prefix
    const bool leaf = eq || lm == 0;
    const uint64_t L = ballot((lm >> rk) & 1ull);  // the left items
    const uint64_t R = S & ~L;
    const int cl = __builtin_popcountll(L), cr = cn - cl, d1 = d + 1;
    const bool lleaf = cl < 2 || d1 >= maxDepth, rleaf = cr < 2 || d1 >= maxDepth;
    put(node, leaf ? (uint32_t)cn << 2 : dim + 1u, leaf ? 0u : __float_as_uint(split));
    put(nn, (uint32_t)cl << 2, 0u);      // the left child as a leaf (real when !leaf && lleaf)
    put(nn + 1, (uint32_t)cr << 2, 0u);  // the right child as a leaf (real when both leaves)
    if (!leaf && R == 0) {  // empty right range: Node::Build fails
      bad = 1;
      break;
    }
    if (lane == 0 && !leaf && lleaf) set_right(nodes, node, nn + 1);
    // push the right child when the left one is walked next (case "descend")
    const bool descend = !leaf && !lleaf;
    writelane(q0, (int)(uint32_t)R, ssp);
    writelane(q1, (int)(uint32_t)(R >> 32), ssp);
    writelane(q2, d1 | (rleaf ? 256 : 0), ssp);
    writelane(q3, node, ssp);
    ssp += descend ? 1 : 0;
    const bool goright = !leaf && lleaf && !rleaf;
    const int nn0 = nn;
    nn += leaf ? 0 : (lleaf ? 2 : 1);
    S = descend ? L : R;
    cn = descend ? cl : cr;
    d = d1;
    node = descend ? nn0 : nn0 + 1;
    if (descend || goright) continue;
    // pop: the next pending right child that is not a leaf (leaves recorded on the way)
    bool found = false;
    while (ssp > 0) {
      ssp--;
      const int e = __builtin_amdgcn_readlane(q2, ssp);
      const int par = __builtin_amdgcn_readlane(q3, ssp);
      S = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(q0, ssp) |
          ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(q1, ssp) << 32);
      if (lane == 0) set_right(nodes, par, nn);
      node = nn++;
      d = e & 255;
      cn = __builtin_popcountll(S);
      if (e & 256) {
        put(node, (uint32_t)cn << 2, 0u);
        continue;
      }
      found = true;
      break;
    }
    if (!found) break;
  }
  return bad;
}

__device__ __forceinline__ int rank_subtree(WaveRng& g, int kx, int ky, int kz, int cnt, int depth, int maxDepth,
                                            int me, int& nn, uint2* nodes) {
  return rank_build(g, rank_prep(kx, ky, kz, cnt), cnt, depth, maxDepth, me, nn, nodes);
}

}  // namespace eao
