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

// ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12)
// (src/ORBmatcher.cc:522-655; LoopClosing::ComputeSim3, src/LoopClosing.cc:265): the same node
// walk as the KeyFrame -> Frame search, but the second side's map points are checked too
// (vpMapPoints2[idx2] && !isBad(), :576-580), its matched flags are vbMatched2 (:534, set at
// :599, never cleared by the rotation check), the distance bar is strict (bestDist1 < TH_LOW,
// :594, against <= in the KeyFrame -> Frame search), the result is indexed by the first side
// (vpMatches12[idx1], :598) and the rotation histogram holds idx1 (:607-613, rot = angle1 -
// angle2). match12[i1] = the KF2 feature whose map point matched KF1 feature i1 (-1 none).
extern "C" int orc_search_by_bow_kf(float nnratio, int check_ori, int n1, const orc_keypoint* kps1,
                                    const uint8_t* desc1, const uint8_t* valid1, int nn1, const int32_t* ids1,
                                    const int32_t* start1, const int32_t* feats1, int n2, const orc_keypoint* kps2,
                                    const uint8_t* desc2, const uint8_t* valid2, int nn2, const int32_t* ids2,
                                    const int32_t* start2, const int32_t* feats2, int32_t* match12) {
  for (int i = 0; i < n1; i++) match12[i] = -1;
  std::vector<char> matched2(n2 > 0 ? n2 : 1, 0);
  int nmatches = 0;
  std::vector<int> rotHist[HISTO_LENGTH];
  const float factor = 1.0f / HISTO_LENGTH;
  int a = 0, b = 0;
  while (a < nn1 && b < nn2) {
    if (ids1[a] == ids2[b]) {
      for (int p = start1[a]; p < start1[a + 1]; p++) {
        const int idx1 = feats1[p];
        if (!valid1[idx1]) continue;  // !pMP1 || pMP1->isBad()
        const uint8_t* d1 = desc1 + 32 * (size_t)idx1;
        int bestDist1 = 256, bestIdx2 = -1, bestDist2 = 256;
        for (int q = start2[b]; q < start2[b + 1]; q++) {
          const int idx2 = feats2[q];
          if (matched2[idx2] || !valid2[idx2]) continue;
          const int dist = hamming(d1, desc2 + 32 * (size_t)idx2);
          if (dist < bestDist1) {
            bestDist2 = bestDist1;
            bestDist1 = dist;
            bestIdx2 = idx2;
          } else if (dist < bestDist2) {
            bestDist2 = dist;
          }
        }
        if (bestDist1 < TH_LOW && (float)bestDist1 < nnratio * (float)bestDist2) {
          match12[idx1] = bestIdx2;
          matched2[bestIdx2] = 1;
          if (check_ori) {
            float rot = kps1[idx1].angle - kps2[bestIdx2].angle;
            if (rot < 0.0) rot += 360.0f;
            int bin = (int)std::round(rot * factor);
            if (bin == HISTO_LENGTH) bin = 0;
            rotHist[bin].push_back(idx1);
          }
          nmatches++;
        }
      }
      a++;
      b++;
    } else if (ids1[a] < ids2[b]) {
      a = (int)(std::lower_bound(ids1 + a, ids1 + nn1, ids2[b]) - ids1);
    } else {
      b = (int)(std::lower_bound(ids2 + b, ids2 + nn2, ids1[a]) - ids2);
    }
  }
  if (check_ori) {
    int i1 = -1, i2 = -1, i3 = -1;
    three_maxima(rotHist, i1, i2, i3);
    for (int i = 0; i < HISTO_LENGTH; i++) {
      if (i == i1 || i == i2 || i == i3) continue;
      for (int j : rotHist[i]) {
        match12[j] = -1;
        nmatches--;
      }
    }
  }
  return nmatches;
}
