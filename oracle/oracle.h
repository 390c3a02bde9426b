/*
 * oracle.h -- CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This library is the parity checker for the MI355X engine. It is linked or
 * loaded ONLY by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg. The product (eao-slam_amd/, include/eao_accel.h) never links it.
 *
 * Parity status: PINNED by in-repo constants only (pattern table, umax, quotas,
 * Hamming SWAR, thresholds, t-table, iForest constants, libstdc++-11 RNG
 * streams); the original binary cannot be built or executed here (SURVEY.md
 * section 8c: OpenCV/Eigen absent, the vendored OpenCV 2.4.5 .so may not be
 * loaded). Where the reference delegates arithmetic to OpenCV 3.2 / Eigen 3.2 /
 * libstdc++ this file restates the published scalar semantics; every such
 * place names the reference call site. Divergences from a SIMD/IPP-dispatched
 * OpenCV build are "parity unpinned" (DESIGN.md, section Oracle).
 */
#ifndef EAO_ORACLE_H
#define EAO_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* mirrors cv::KeyPoint field order (28 bytes) */
typedef struct {
  float x, y, size, angle, response;
  int32_t octave, class_id;
} orc_keypoint;

/* ---- ORB extractor (reference src/ORBextractor.cc) ---- */
int orc_orb_params(int nfeatures, float scale_factor, int nlevels,
                   float* scale, float* inv_scale, float* sigma2, float* inv_sigma2,
                   int* feats_per_level, int* umax16);
/* level sizes of the pyramid (w,h per level) */
int orc_orb_level_sizes(int w, int h, float scale_factor, int nlevels, int* sizes);
/* compute pyramid; out = concatenation of levels, each w_l*h_l bytes, tightly packed */
int orc_orb_pyramid(const uint8_t* img, int w, int h, float scale_factor, int nlevels, uint8_t* out);
/* FAST candidates of one level before quadtree distribution, in
   vToDistributeKeys order (coordinates relative to minBorder like the reference) */
int orc_orb_level_candidates(const uint8_t* level, int w, int h, int iniTh, int minTh,
                             orc_keypoint* out, int cap, int* n_out);
/* 7x7 sigma=2 REFLECT_101 blur (8U fixed-point path) */
int orc_gaussian_blur7(const uint8_t* src, int w, int h, uint8_t* dst);
float orc_fast_atan2(float y, float x);
/* cvtColor(CV_{RGB,BGR}[A]2GRAY) (OpenCV 3.2 RGB2Gray<uchar>); rgb: the RGB codes */
int orc_color_to_gray(const uint8_t* src, int w, int h, int pitch, int cn, int rgb, uint8_t* dst);
/* full ORBextractor::operator() */
int orc_orb_extract(const uint8_t* img, int w, int h, int nfeatures, float scale_factor,
                    int nlevels, int iniTh, int minTh,
                    orc_keypoint* kps, uint8_t* desc, int cap, int* n_out);

/* ---- Frame grid / matcher (reference src/Frame.cc, src/ORBmatcher.cc) ---- */
int orc_descriptor_distance(const uint8_t* a, const uint8_t* b);

typedef struct {
  int img_w, img_h;          /* image bounds (mnMinX=0,mnMaxX=w,...) */
  float fx, fy, cx, cy;
} orc_camera;

/* SearchByProjection(CurrentFrame, LastFrame, th, bMono=true), ORBmatcher.cc:1328-1470.
   last frame: n_last keypoints, last_has_mp[i] (0/1, non-outlier map point present),
   last_mp_pos[3*i] world position, last_mp_desc[32*i] map-point descriptor.
   current frame: n_cur keypoints + descriptors.  Tcw 4x4 row-major float (current pose).
   Output: cur_match[n_cur] = index of last-frame keypoint whose MP was assigned, -1 none.
   Returns nmatches. */
int orc_search_by_projection_motion(const orc_camera* cam, const float* Tcw, float th, int check_ori,
                                    int n_last, const orc_keypoint* last_kps,
                                    const uint8_t* last_has_mp, const float* last_mp_pos,
                                    const uint8_t* last_mp_desc,
                                    int n_cur, const orc_keypoint* cur_kps, const uint8_t* cur_desc,
                                    int nlevels, const float* scale_factors,
                                    int32_t* cur_match);
/* bench.py's all-cores CPU baseline leg (baseline_mt.cpp): frame-parallel extraction of
   n frames, then the motion search of every pair (t-1, t), over `threads` std::threads */
double orc_extract_match_mt(const uint8_t* frames, int n, int w, int h, int nfeatures, float scale_factor,
                            int nlevels, int iniTh, int minTh, const orc_camera* cam, const float* Tcw,
                            const uint8_t* has, const float* mpos, float th, int check_ori, const float* scales,
                            int cap, int threads, orc_keypoint* kps, uint8_t* desc, int* nkp, int32_t* match,
                            int* nmatch);

/* SearchByProjection(Frame&, vector<MapPoint*>, th), ORBmatcher.cc:45-129, for map
   points already passed through isInFrustum (track_* inputs, Frame.cc:390-446). */
int orc_search_by_projection_local(const orc_camera* cam, float th, float nnratio,
                                   int n_mp, const uint8_t* in_view, const float* proj_xy,
                                   const int32_t* pred_level,
                                   const float* view_cos, const uint8_t* mp_desc,
                                   int n_cur, const orc_keypoint* cur_kps, const uint8_t* cur_desc,
                                   const int32_t* cur_preassigned,
                                   int nlevels, const float* scale_factors,
                                   int32_t* cur_match);

/* isInFrustum + PredictScale for a batch of map points */
int orc_is_in_frustum(const orc_camera* cam, const float* Tcw, int n_mp, const float* mp_pos,
                      const float* mp_normal, const float* mp_min_dist, const float* mp_max_dist,
                      float view_cos_limit, float log_scale_factor,
                      uint8_t* in_view, float* proj_xy, int32_t* pred_level, float* view_cos);

/* SearchByProjection(Frame&, KeyFrame*, set<MapPoint*>, th, ORBdist), ORBmatcher.cc:1472-1599
   (relocalisation). kf_mp_valid[i] = MP present, not bad, not already found. */
int orc_search_by_projection_keyframe(const orc_camera* cam, const float* Tcw, float th,
                                      int orb_dist, int check_ori, int n_kf,
                                      const orc_keypoint* kf_kps, const uint8_t* kf_mp_valid,
                                      const float* kf_mp_pos, const uint8_t* kf_mp_desc,
                                      const float* kf_mp_min_dist, const float* kf_mp_max_dist,
                                      float log_scale_factor, int n_cur,
                                      const orc_keypoint* cur_kps, const uint8_t* cur_desc,
                                      const int32_t* cur_preassigned, int nlevels,
                                      const float* scale_factors, int32_t* cur_match);

/* SearchForInitialization, ORBmatcher.cc:405-520 */
int orc_search_for_initialization(const orc_camera* cam, float nnratio, int check_ori,
                                  int n1, const orc_keypoint* kps1, const uint8_t* desc1,
                                  int n2, const orc_keypoint* kps2, const uint8_t* desc2,
                                  float* prev_matched_xy, int window,
                                  int32_t* matches12);

/* ---- EAO association (reference src/Object.cc, include/isolation_forest.h) ---- */
typedef struct {
  int32_t verdict;            /* 0: m<20 (break), 1: pass, 2: fail */
  int32_t m, n;               /* valid frame points, sampled object points */
  float w[3];                 /* rank sums W_x,W_y,W_z */
  float r1, r2;               /* acceptance bounds */
  float cnt_gt[3], cnt_lt[3], cnt_eq[3];
} orc_np_stats;

/* NoParaDataAssociation, Object.cc:714-930. valid flags mark !isBad && !out_point.
   n_total = object list size (including invalid), used by the subsampling step. */
int orc_np_test(int m_total, const float* frame_pts, const uint8_t* frame_valid,
                int n_total, const float* obj_pts, const uint8_t* obj_valid,
                orc_np_stats* out);

/* IsolationForest (isolation_forest.h) as used by Object.cc:1202-1309:
   Build(trees, seed, data, sampleSize) + GetAnomalyScores. */
int orc_iforest_scores(const float* pts, int n, uint32_t trees, uint32_t seed,
                       uint32_t sample_size, double* scores);

/* mt19937 / libstdc++-11 distribution KATs */
void orc_mt19937_stream(uint32_t seed, int n, uint32_t* out);
uint32_t orc_lemire_u32(uint32_t seed, int n_draws, uint32_t range, uint32_t* out);
int orc_shuffle_ids(uint32_t seed, int n, uint32_t* ids);
void orc_canonical_float(uint32_t seed, int n, float lo, float hi, float* out);

/* Converter::bboxOverlapratio* (Converter.cc:194-212); rects are int[4] x,y,w,h */
float orc_bbox_iou(const int* r1, const int* r2);
float orc_bbox_former(const int* r1, const int* r2);
float orc_bbox_latter(const int* r1, const int* r2);

/* ComputeProjectRectFrame, Object.cc:1558-1603 -> rect int[4] */
int orc_project_rect(const orc_camera* cam, const float* Tcw, int n, const float* pts, int* rect);

/* deterministic association replay -- see assoc_ref.cpp */
typedef struct orc_replay orc_replay;
orc_replay* orc_replay_create(const char* flag, int img_w, int img_h, const float* K4);
void orc_replay_destroy(orc_replay* r);
/* one frame: pose, boxes[k*5]={class,x,y,w,h} (file order), tracked points */
int orc_replay_frame(orc_replay* r, int frame_id, const float* Tcw,
                     int n_boxes, const int32_t* boxes,
                     int n_pts, const int32_t* mp_ids, const float* mp_pos, const float* kp_uv,
                     const uint8_t* mp_bad,
                     int32_t* det_out /* n_boxes*4: outcome, obj id, class, npoints */);
int orc_replay_local_mapping(orc_replay* r);
/* map-point changes of LocalMapping (BA positions, culling / replacement as bad flags) for
   the points with the given ids; pos (n x 3) or bad (n) may be NULL to leave that field */
int orc_replay_update_points(orc_replay* r, int n, const int32_t* ids, const float* pos, const uint8_t* bad);
int orc_replay_num_objects(orc_replay* r);
/* per object summary: id, class, bad, nframes, npts, center[3], std[3], cstd[3],
   cuboid extents lenth/width/height, rmax, last_add, rect_project[4] */
int orc_replay_object(orc_replay* r, int i, int32_t* ints /*8*/, float* floats /*20*/);
/* frame line segments (Frame::all_lines_eigen rows x1,y1,x2,y2) for the next n_frames
   orc_replay_frame calls, consumed one set per frame */
int orc_replay_lines(orc_replay* r, int n_frames, const int32_t* n_lines, const float* lines);
int orc_replay_object_points(orc_replay* r, int i, int32_t* ids, int cap);

/* per-frame line detection (lines_ref.cpp): GaussianBlur 5x5 sigma 1 + EDLine maps,
   edge chains, and detect_raw_lines + filter_lines output (startX, startY, endX, endY,
   angle, lineLength) per kept line */
int orc_line_maps(const uint8_t* gray, int w, int h, uint8_t* blur, int16_t* dx, int16_t* dy, int16_t* g,
                  uint8_t* dir);
int orc_edge_chains(const uint8_t* gray, int w, int h, uint32_t* xy, int cap_px, uint32_t* sid, int cap_edges,
                    int* n_px, int* n_edges);
/* the restatement under other EDLineDetector knobs (ip = grad th, anchor th, scan, min line
   length, gradient divisor, validate): kept chains as a 255/0 map, and EDline's raw segments -- only for
   pinning against the Edge Drawing library's outputs (tests/test_oracle_ed_pin.py) */
int orc_ed_edge_map(const uint8_t* gray, int w, int h, const int* ip, double fit_err, uint8_t* map, int* n_chains);
int orc_ed_segments(const uint8_t* gray, int w, int h, const int* ip, double fit_err, float* out, int cap,
                    int* n_out);
int orc_edlines(const uint8_t* gray, int w, int h, float min_length, float* out, int cap, int* n_out);
/* the same on the colour frame BinaryDescriptor::detectImpl receives: cn = 3 / 4 bytes per pixel
   converted with COLOR_BGR2GRAY first (binary_descriptor.cpp:490-495); cn = 1 is gray */
int orc_edlines_color(const uint8_t* img, int w, int h, int pitch, int cn, float min_length, float* out, int cap,
                      int* n_out);

/* ---- Optimizer::PoseOptimization, monocular edges (src/Optimizer.cc:243-457) ----
   Tcw 4x4 row-major float (pFrame->mTcw); kps = mvKeysUn; has_mp[i] = mvpMapPoints[i] != 0;
   mp_pos = GetWorldPos(); outlier[i] (mvbOutlier) written where has_mp[i]. */
int orc_pose_optimization(const orc_camera* cam, const float* Tcw_in, int n,
                          const orc_keypoint* kps, const uint8_t* has_mp, const float* mp_pos,
                          const float* inv_level_sigma2, float* Tcw_out, uint8_t* outlier,
                          int* n_inliers);

/* ---- BoW (src/Frame.cc:516-523 -> DBoW2 TemplatedVocabulary::transform, TF_IDF + L1) and
   ORBmatcher::SearchByBoW(KeyFrame*, Frame&) (src/ORBmatcher.cc:159-288). Vocabulary as arrays:
   node descriptors [n][32], parent [n] (root 0: -1), word id [n] (-1: inner node), weight [n].
   FeatureVector as CSR: node_ids ascending, node_start [nn + 1], node_feats. f_match[iF] = the
   keyframe feature whose map point matched (-1 none). */
void* orc_vocab_create(int n_nodes, const uint8_t* node_desc, const int32_t* parent,
                       const int32_t* word_id, const double* weight, int L);
void orc_vocab_destroy(void* v);
int orc_bow_transform(void* voc, int n, const uint8_t* desc, int levelsup, int32_t* word_ids,
                      double* word_weights, int* n_words, int32_t* node_ids, int32_t* node_start,
                      int32_t* node_feats, int* n_fnodes);
int orc_search_by_bow(float nnratio, int check_ori, int n_kf, const orc_keypoint* kf_kps,
                      const uint8_t* kf_desc, const uint8_t* kf_mp_valid, int kf_nn,
                      const int32_t* kf_node_ids, const int32_t* kf_node_start,
                      const int32_t* kf_node_feats, int n_f, const orc_keypoint* f_kps,
                      const uint8_t* f_desc, int f_nn, const int32_t* f_node_ids,
                      const int32_t* f_node_start, const int32_t* f_node_feats, int32_t* f_match);

/* ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>&) (src/ORBmatcher.cc:522-655):
   valid1 / valid2 = GetMapPointMatches()[i] && !isBad(); match12[i1] = matched KF2 feature (-1 none) */
int orc_search_by_bow_kf(float nnratio, int check_ori, int n1, const orc_keypoint* kps1, const uint8_t* desc1,
                         const uint8_t* valid1, int nn1, const int32_t* ids1, const int32_t* start1,
                         const int32_t* feats1, int n2, const orc_keypoint* kps2, const uint8_t* desc2,
                         const uint8_t* valid2, int nn2, const int32_t* ids2, const int32_t* start2,
                         const int32_t* feats2, int32_t* match12);

#ifdef __cplusplus
}
#endif
#endif
