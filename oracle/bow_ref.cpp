/*
 * bow_ref.cpp -- CPU restatement of the BoW path of tracking (TEST INFRASTRUCTURE ONLY):
 *   Frame::ComputeBoW -> TemplatedVocabulary::transform(features, BowVector, FeatureVector, 4)
 *     (src/Frame.cc:516-523; Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1139-1206, 1230-1271,
 *      BowVector::addWeight / normalize(L1) BowVector.cpp, FeatureVector::addFeature
 *      FeatureVector.cpp), for the ORB vocabulary's TF_IDF weighting + L1 scoring
 *     (loadFromTextFile header "k L 0 0");
 *   ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&) (src/ORBmatcher.cc:159-288)
 *     with ComputeThreeMaxima (:1601-1642).
 * The vocabulary is an input (node descriptors, parents, word ids, weights): the reference's
 * Vocabulary/ORBvoc.bin is a missing blob, so tests use synthetic trees.
 */
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <vector>
#include "oracle.h"

namespace {

int hamming(const uint8_t* a, const uint8_t* b) {  // FORB::distance / DescriptorDistance
  int d = 0;
  for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
  return d;
}

struct Vocab {
  int L = 0;
  std::vector<std::vector<int>> children;
  const uint8_t* desc = nullptr;
  const int32_t* word = nullptr;
  const double* weight = nullptr;
  bool empty = true;
};

// transform(feature, word_id, weight, &nid, levelsup) (TemplatedVocabulary.h:1230-1271)
void transform1(const Vocab& V, const uint8_t* f, int levelsup, int& word, double& w, int& nid) {
  const int nid_level = V.L - levelsup;
  if (nid_level <= 0) nid = 0;
  int fid = 0, level = 0;
  do {
    ++level;
    const std::vector<int>& ch = V.children[fid];
    fid = ch[0];
    int best = hamming(f, V.desc + 32 * (size_t)fid);
    for (size_t c = 1; c < ch.size(); c++) {
      const int d = hamming(f, V.desc + 32 * (size_t)ch[c]);
      if (d < best) {
        best = d;
        fid = ch[c];
      }
    }
    if (level == nid_level) nid = fid;
  } while (!V.children[fid].empty());
  word = V.word[fid];
  w = V.weight[fid];
}

const int TH_LOW = 50, HISTO_LENGTH = 30;  // ORBmatcher.cc:37-39

void three_maxima(const std::vector<int>* h, int& ind1, int& ind2, int& ind3) {
  int max1 = 0, max2 = 0, max3 = 0;
  for (int i = 0; i < HISTO_LENGTH; i++) {
    const int s = (int)h[i].size();
    if (s > max1) {
      max3 = max2;
      max2 = max1;
      max1 = s;
      ind3 = ind2;
      ind2 = ind1;
      ind1 = i;
    } else if (s > max2) {
      max3 = max2;
      max2 = s;
      ind3 = ind2;
      ind2 = i;
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

}  // namespace

// the vocabulary as loadFromTextFile leaves it: children in file (id) order; the arrays are
// the caller's and must outlive the handle
extern "C" void* orc_vocab_create(int n_nodes, const uint8_t* node_desc, const int32_t* parent,
                                  const int32_t* word_id, const double* weight, int L) {
  Vocab* V = new Vocab();
  V->L = L;
  V->children.resize(n_nodes);
  for (int i = 1; i < n_nodes; i++) V->children[parent[i]].push_back(i);
  V->desc = node_desc;
  V->word = word_id;
  V->weight = weight;
  bool any_word = false;
  for (int i = 0; i < n_nodes; i++) any_word |= word_id[i] >= 0;
  V->empty = !any_word || n_nodes < 2 || V->children[0].empty();
  return V;
}
extern "C" void orc_vocab_destroy(void* v) { delete (Vocab*)v; }

extern "C" int orc_bow_transform(void* voc, int n, const uint8_t* desc, int levelsup, int32_t* word_ids,
                                 double* word_weights, int* n_words, int32_t* node_ids,
                                 int32_t* node_start, int32_t* node_feats, int* n_fnodes) {
  const Vocab& V = *(const Vocab*)voc;
  std::map<int, double> bow;                 // BowVector
  std::map<int, std::vector<int>> fv;        // FeatureVector
  if (!V.empty) {
    for (int i = 0; i < n; i++) {
      int w, nid = 0;
      double wt;
      transform1(V, desc + 32 * (size_t)i, levelsup, w, wt, nid);
      if (wt > 0) {
        auto it = bow.find(w);
        if (it != bow.end()) it->second += wt;
        else bow.insert({w, wt});
        fv[nid].push_back(i);
      }
    }
    double norm = 0.0;  // normalize(L1)
    for (auto& kv : bow) norm += std::fabs(kv.second);
    if (norm > 0.0)
      for (auto& kv : bow) kv.second /= norm;
  }
  int k = 0;
  for (auto& kv : bow) {
    word_ids[k] = kv.first;
    word_weights[k] = kv.second;
    k++;
  }
  *n_words = k;
  k = 0;
  int p = 0;
  for (auto& kv : fv) {
    node_ids[k] = kv.first;
    node_start[k] = p;
    for (int f : kv.second) node_feats[p++] = f;
    k++;
  }
  node_start[k] = p;
  *n_fnodes = k;
  return 0;
}

extern "C" int orc_search_by_bow(float nnratio, int check_ori, int n_kf, const orc_keypoint* kf_kps,
                                 const uint8_t* kf_desc, const uint8_t* kf_mp_valid, int kf_nn,
                                 const int32_t* kf_node_ids, const int32_t* kf_node_start,
                                 const int32_t* kf_node_feats, int n_f, const orc_keypoint* f_kps,
                                 const uint8_t* f_desc, int f_nn, const int32_t* f_node_ids,
                                 const int32_t* f_node_start, const int32_t* f_node_feats,
                                 int32_t* f_match) {
  (void)n_kf;
  for (int i = 0; i < n_f; i++) f_match[i] = -1;
  int nmatches = 0;
  std::vector<int> rotHist[HISTO_LENGTH];
  const float factor = 1.0f / HISTO_LENGTH;
  int a = 0, b = 0;
  while (a < kf_nn && b < f_nn) {
    if (kf_node_ids[a] == f_node_ids[b]) {
      for (int p = kf_node_start[a]; p < kf_node_start[a + 1]; p++) {
        const int ikf = kf_node_feats[p];
        if (!kf_mp_valid[ikf]) continue;  // !pMP || pMP->isBad()
        const uint8_t* dKF = kf_desc + 32 * (size_t)ikf;
        int best1 = 256, bestIdx = -1, best2 = 256;
        for (int q = f_node_start[b]; q < f_node_start[b + 1]; q++) {
          const int iF = f_node_feats[q];
          if (f_match[iF] >= 0) continue;
          const int d = hamming(dKF, f_desc + 32 * (size_t)iF);
          if (d < best1) {
            best2 = best1;
            best1 = d;
            bestIdx = iF;
          } else if (d < best2) {
            best2 = d;
          }
        }
        if (best1 <= TH_LOW && (float)best1 < nnratio * (float)best2) {
          f_match[bestIdx] = ikf;
          if (check_ori) {
            float rot = kf_kps[ikf].angle - f_kps[bestIdx].angle;
            if (rot < 0.0) rot += 360.0f;
            int bin = (int)std::round(rot * factor);
            if (bin == HISTO_LENGTH) bin = 0;
            rotHist[bin].push_back(bestIdx);
          }
          nmatches++;
        }
      }
      a++;
      b++;
    } else if (kf_node_ids[a] < f_node_ids[b]) {
      a = (int)(std::lower_bound(kf_node_ids + a, kf_node_ids + kf_nn, f_node_ids[b]) - kf_node_ids);
    } else {
      b = (int)(std::lower_bound(f_node_ids + b, f_node_ids + f_nn, kf_node_ids[a]) - f_node_ids);
    }
  }
  if (check_ori) {
    int i1 = -1, i2 = -1, i3 = -1;
    three_maxima(rotHist, i1, i2, i3);
    for (int i = 0; i < HISTO_LENGTH; i++) {
      if (i == i1 || i == i2 || i == i3) continue;
      for (int j : rotHist[i]) {
        f_match[j] = -1;
        nmatches--;
      }
    }
  }
  return nmatches;
}
