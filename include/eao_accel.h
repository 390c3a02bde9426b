/*
 * eao_accel.h -- C ABI of the MI355X-native EAO-SLAM front-end + object
 * association engine (gfx950, HIP).
 *
 * Plain C: opaque handles, plain pointers and sizes, caller-owned buffers,
 * int status (0 ok, <0 error, see EAO_E_*). No torch / OpenCV / Eigen types.
 * Every entry point names the reference interface it replaces (paths relative
 * to the reference repository yanmin-wu/EAO-SLAM). INTEGRATION.md shows the
 * reference-side shims (ORBextractor::operator(), ORBmatcher::SearchBy*,
 * Object_2D / Object_Map) that bind these symbols so mono_tum links unchanged.
 *
 * Device pointers: functions with the suffix _device take HIP device pointers
 * (inputs resident in HBM) and a hipStream_t passed as void* (NULL = the
 * handle's own stream). All other functions take host pointers.
 *
 * Streams and scratch: a handle's calls (batched or single-frame) use scratch
 * owned by the handle, whatever stream they are given. Calls on one handle must
 * be ordered on one stream (or synchronised by the caller between streams); use
 * one handle per concurrently used stream. Single-frame calls run on the handle's
 * own stream and return after it drains.
 *
 * The engine has NO CPU fallback: without a usable gfx950 device every call
 * returns EAO_E_NODEVICE.
 */
#ifndef EAO_ACCEL_H
#define EAO_ACCEL_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EAO_OK 0
#define EAO_E_ARG (-1)
#define EAO_E_NODEVICE (-2)
#define EAO_E_HIP (-3)
#define EAO_E_CAPACITY (-4)
#define EAO_E_STATE (-5)

/* mirrors cv::KeyPoint {pt.x, pt.y, size, angle, response, octave, class_id}
   (28 bytes, same field order) -- the element type of Frame::mvKeys */
typedef struct {
  float x, y, size, angle, response;
  int32_t octave, class_id;
} eao_keypoint;

/* ORB parameters: ORBextractor::ORBextractor(nfeatures, scaleFactor, nlevels,
   iniThFAST, minThFAST) (include/ORBextractor.h:50-51); max_* size the
   handle's HBM workspace (batch of frames of at most max_width x max_height). */
typedef struct {
  int32_t nfeatures;
  float scale_factor;
  int32_t nlevels;
  int32_t ini_th_fast;
  int32_t min_th_fast;
  int32_t width, height; /* frame size the handle is planned for */
  int32_t max_batch;     /* frames per batched call */
} eao_orb_params;

typedef struct eao_orb eao_orb;

/* library / device */
const char* eao_version(void);
int eao_device_ok(int device); /* 1 when a gfx950 device is usable */
const char* eao_last_error(void);

/* --- ORB extraction: replaces ORBextractor (src/ORBextractor.cc:410-1132) --- */
/* ctor, src/ORBextractor.cc:410-470 */
int eao_orb_create(const eao_orb_params* p, int device, eao_orb** out);
int eao_orb_destroy(eao_orb* h);
/* GetScaleFactors/GetInverseScaleFactors/GetScaleSigmaSquares/
   GetInverseScaleSigmaSquares (include/ORBextractor.h:63-83); arrays of nlevels */
int eao_orb_scale_tables(const eao_orb* h, float* scale, float* inv_scale, float* sigma2,
                         float* inv_sigma2);
/* per-level feature quotas mnFeaturesPerLevel (src/ORBextractor.cc:435-446) */
int eao_orb_level_quotas(const eao_orb* h, int32_t* quotas);
/* output capacity (keypoints) per frame slot of the batched API */
int eao_orb_frame_capacity(const eao_orb* h);
/* ORBextractor::operator()(image, mask, keypoints, descriptors)
   (src/ORBextractor.cc:1043-1105) on one host image. Keypoints in the
   reference order (level 0..7, quadtree order within a level); desc = n x 32
   bytes. An empty image (w*h == 0) returns n_out = 0 like the reference's
   early return; 0 keypoints means "descriptors.release()". */
int eao_orb_extract(eao_orb* h, const uint8_t* gray, int w, int h_, int stride,
                    eao_keypoint* kps, uint8_t* desc, int cap, int* n_out);
/* batched, HBM-resident: frames [n][h][pitch] u8 device; outputs per frame slot
   f: kps[f*cap .. f*cap+counts[f]), desc[(f*cap+i)*32], counts[f]. cap must be
   >= eao_orb_frame_capacity(). */
int eao_orb_extract_batch_device(eao_orb* h, const uint8_t* d_frames, int nframes, int pitch,
                                 eao_keypoint* d_kps, uint8_t* d_desc, int32_t* d_counts, int cap,
                                 void* stream);
/* per-stage timing of the batched path (HIP events on the launch stream):
   enable once, then after a run eao_orb_stage_ms writes min(n, 4) values in
   ms -- pyramid (7 resizes), FAST cells, quadtree distribution, orient + blur +
   describe (the level blur is fused into the descriptor kernel) -- and returns the
   number of stages (4). */
int eao_orb_set_timing(eao_orb* h, int on);
int eao_orb_stage_ms(eao_orb* h, float* ms, int n);
/* debug taps for parity tests (device work, host results) */
int eao_orb_debug_pyramid(eao_orb* h, const uint8_t* gray, uint8_t* out /* concatenated levels */);

/* --- frame input stage: cvtColor(mImGray, mImGray, CV_RGB2GRAY / CV_BGR2GRAY /
   CV_RGBA2GRAY / CV_BGRA2GRAY) of Tracking::GrabImageMonocular (src/Tracking.cc:349-362),
   OpenCV 3.2's fixed-point RGB2Gray<uchar>, for a batch of HBM-resident frames:
   d_color [n][h][pitch] with `channels` (3 or 4) interleaved u8 per pixel; rgb = mbRGB
   (Camera.RGB: 1 applies the RGB code to imread's BGR bytes); d_gray
   [n][h][gray_pitch]. stream = HIP stream (NULL: the default stream). --- */
int eao_color_to_gray_batch_device(const uint8_t* d_color, int nframes, int w, int h, int pitch, int channels,
                                   int rgb, uint8_t* d_gray, int gray_pitch, int device, void* stream);

/* --- matching: replaces ORBmatcher (src/ORBmatcher.cc) + Frame grid ---------- */
typedef struct {
  int32_t img_w, img_h; /* Frame::mnMinX=0..mnMaxX=w, mnMinY=0..mnMaxY=h (k1 == 0) */
  float fx, fy, cx, cy;
} eao_camera;

typedef struct eao_matcher eao_matcher;
int eao_matcher_create(int device, int max_kps, int max_batch, eao_matcher** out);
int eao_matcher_destroy(eao_matcher* m);

/* DescriptorDistance (src/ORBmatcher.cc:1647-1663) for candidate lists:
   dist[i] = hamming(q[qidx[i]], t[tidx[i]]) -- host arrays, GPU compute */
int eao_hamming_pairs(eao_matcher* m, const uint8_t* q, int nq, const uint8_t* t, int nt,
                      const int32_t* qidx, const int32_t* tidx, int npairs, int32_t* dist);

/* SearchByProjection(CurrentFrame, LastFrame, th, bMono=true)
   (src/ORBmatcher.cc:1328-1470) with the Frame grid (src/Frame.cc:351-513).
   last_has_mp[i]: LastFrame.mvpMapPoints[i] && !mvbOutlier[i]; last_mp_pos /
   last_mp_desc: that map point's GetWorldPos() / GetDescriptor().
   cur_match[i2] = index i of the last-frame keypoint whose map point was
   assigned to current keypoint i2, -1 if none. Returns nmatches (>= 0). */
int eao_match_motion(eao_matcher* m, const eao_camera* cam, const float* Tcw, float th,
                     int check_ori, int n_last, const eao_keypoint* last_kps,
                     const uint8_t* last_has_mp, const float* last_mp_pos,
                     const uint8_t* last_mp_desc, int n_cur, const eao_keypoint* cur_kps,
                     const uint8_t* cur_desc, int nlevels, const float* scale_factors,
                     int32_t* cur_match);

/* batched motion-model search, HBM-resident: pair p matches frame slot p+1
   (current) against slot p (last) for p in [0, nframes-1). Frame slot arrays
   are [nframes][cap] (kps, desc*32, has_mp, mp_pos*3, mp_desc*32); Tcw[nframes][16].
   cur_match[(p+1)*cap + i2], nmatches[p+1]. */
int eao_match_motion_batch_device(eao_matcher* m, const eao_camera* cam, int nframes, int cap,
                                  const float* d_Tcw, float th, int check_ori,
                                  const eao_keypoint* d_kps, const uint8_t* d_desc,
                                  const int32_t* d_counts, const uint8_t* d_has_mp,
                                  const float* d_mp_pos, const uint8_t* d_mp_desc, int nlevels,
                                  const float* scale_factors, int32_t* d_cur_match,
                                  int32_t* d_nmatches, void* stream);

/* Frame::isInFrustum (src/Frame.cc:390-446) + MapPoint::PredictScale
   (src/MapPoint.cc:385-394) for a batch of map points. */
int eao_is_in_frustum(eao_matcher* m, const eao_camera* cam, const float* Tcw, int n_mp,
                      const float* mp_pos, const float* mp_normal, const float* mp_min_dist,
                      const float* mp_max_dist, float view_cos_limit, float log_scale_factor,
                      uint8_t* in_view, float* proj_xy, int32_t* pred_level, float* view_cos);

/* SearchByProjection(Frame&, const vector<MapPoint*>&, th)
   (src/ORBmatcher.cc:45-129). in_view[i] = mbTrackInView (isInFrustum);
   pred_level is clamped to [0, nlevels-1].
   cur_preassigned[i] >= 0 marks keypoints that already hold a map point. */
int eao_match_local(eao_matcher* m, const eao_camera* cam, float th, float nnratio, int n_mp,
                    const uint8_t* in_view, const float* proj_xy, const int32_t* pred_level,
                    const float* view_cos,
                    const uint8_t* mp_desc, int n_cur, const eao_keypoint* cur_kps,
                    const uint8_t* cur_desc, const int32_t* cur_preassigned, int nlevels,
                    const float* scale_factors, int32_t* cur_match);

/* SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>& sAlreadyFound, th, ORBdist)
   (src/ORBmatcher.cc:1472-1599; relocalisation, src/Tracking.cc:2295,2309).
   Keyframe side: kf_kps (angles for the rotation check), kf_mp_valid[i] = vpMPs[i] &&
   !isBad() && !sAlreadyFound.count(vpMPs[i]), positions / descriptors and
   mfMinDistance / mfMaxDistance of those map points. cur_preassigned[i2] >= 0 marks
   CurrentFrame.mvpMapPoints[i2] already set (kept in cur_match). New matches write the
   keyframe index i into cur_match[i2]. PredictScale is clamped.
   Returns nmatches. */
int eao_match_keyframe(eao_matcher* m, const eao_camera* cam, const float* Tcw, float th,
                       int orb_dist, int check_ori, int n_kf, const eao_keypoint* kf_kps,
                       const uint8_t* kf_mp_valid, const float* kf_mp_pos,
                       const uint8_t* kf_mp_desc, const float* kf_mp_min_dist,
                       const float* kf_mp_max_dist, float log_scale_factor, int n_cur,
                       const eao_keypoint* cur_kps, const uint8_t* cur_desc,
                       const int32_t* cur_preassigned, int nlevels, const float* scale_factors,
                       int32_t* cur_match);

/* SearchForInitialization (src/ORBmatcher.cc:405-520); prev_matched_xy is
   updated in place like vbPrevMatched. */
int eao_match_init(eao_matcher* m, const eao_camera* cam, float nnratio, int check_ori, int n1,
                   const eao_keypoint* kps1, const uint8_t* desc1, int n2,
                   const eao_keypoint* kps2, const uint8_t* desc2, float* prev_matched_xy,
                   int window, int32_t* matches12);

/* batched, HBM-resident forms of the three single-frame searches above (same
   arguments per search; no reference counterpart batches them -- the tracker calls
   one per frame, Tracking.cc:1985 (local map), :2295,2309 (relocalisation),
   :1042 (initialisation) -- this is the form a multi-stream / multi-camera caller
   queues). Search f reads query slot f ([nsearch][q_cap] arrays with counts
   d_n_*[f]) and frame slot f ([nsearch][cap] keypoints / descriptors / preassigned
   with counts d_n_cur[f]); outputs are [nsearch][cap] (init: [nsearch][cap1]) plus
   d_nmatches[f]. Keyframe poses d_Tcw are [nsearch][16]. Asynchronous on `stream`
   (NULL: the matcher's own stream). */
int eao_match_local_batch_device(eao_matcher* m, const eao_camera* cam, int nsearch, float th, float nnratio,
                                 int mp_cap, const int32_t* d_n_mp, const uint8_t* d_in_view, const float* d_proj_xy,
                                 const int32_t* d_pred_level, const float* d_view_cos, const uint8_t* d_mp_desc,
                                 int cap, const int32_t* d_n_cur, const eao_keypoint* d_cur_kps,
                                 const uint8_t* d_cur_desc, const int32_t* d_cur_preassigned, int nlevels,
                                 const float* scale_factors, int32_t* d_cur_match, int32_t* d_nmatches,
                                 void* stream);
int eao_match_keyframe_batch_device(eao_matcher* m, const eao_camera* cam, int nsearch, const float* d_Tcw,
                                    float th, int orb_dist, int check_ori, int kf_cap, const int32_t* d_n_kf,
                                    const eao_keypoint* d_kf_kps, const uint8_t* d_kf_mp_valid,
                                    const float* d_kf_mp_pos, const uint8_t* d_kf_mp_desc,
                                    const float* d_kf_mp_min_dist, const float* d_kf_mp_max_dist,
                                    float log_scale_factor, int cap, const int32_t* d_n_cur,
                                    const eao_keypoint* d_cur_kps, const uint8_t* d_cur_desc,
                                    const int32_t* d_cur_preassigned, int nlevels, const float* scale_factors,
                                    int32_t* d_cur_match, int32_t* d_nmatches, void* stream);
int eao_match_init_batch_device(eao_matcher* m, const eao_camera* cam, int nsearch, float nnratio, int check_ori,
                                int cap1, const int32_t* d_n1, const eao_keypoint* d_kps1, const uint8_t* d_desc1,
                                int cap2, const int32_t* d_n2, const eao_keypoint* d_kps2, const uint8_t* d_desc2,
                                float* d_prev_matched_xy, int window, int32_t* d_matches12, int32_t* d_nmatches,
                                void* stream);

/* --- per-frame line detection: replaces line_lbd_detect::detect_raw_lines +
   filter_lines (src/Frame.cc:324-328; src/line_detect/line_lbd_allclass.cpp:137-214)
   with the tracker's single octave (Tracking.cc:161-163): GaussianBlur(5x5, sigma 1),
   EDLineDetector::EDline (src/line_detect/libs/binary_descriptor.cpp:1583-2906) and the
   keyline endpoint ordering of OctaveKeyLines (:866-887, 1073-1141). A line is
   (startX, startY, endX, endY, angle, lineLength) -- keylines_to_mat's four columns
   plus KeyLine::angle / lineLength -- kept when lineLength > min_length (50 in the
   reference). --------------------------------------------------------------------- */
typedef struct eao_lines eao_lines;
int eao_lines_create(int device, int width, int height, int max_batch, eao_lines** out);
int eao_lines_destroy(eao_lines* l);
/* batched, HBM-resident: gray frames [n][height][pitch] u8; d_lines [n][cap][6] f32,
   d_counts[n] (the frame's line count, > cap when truncated; -1 when the reference's
   EdgeDrawing would fail: more anchors / edge pixels / edges than its arrays hold) */
int eao_lines_detect_batch_device(eao_lines* l, const uint8_t* d_gray, int nframes, int pitch, float min_length,
                                  float* d_lines, int32_t* d_counts, int cap, void* stream);
/* one host frame; returns EAO_E_CAPACITY when more than cap lines (n_out holds the count) */
int eao_lines_detect(eao_lines* l, const uint8_t* gray, int pitch, float min_length, float* lines, int cap,
                     int* n_out);
/* BinaryDescriptor::detectImpl's own input: the colour frame the EAO Frame ctor hands to
   detect_raw_lines (rawImage, src/Frame.cc:324; src/Tracking.cc:340,389), channels = 3 or 4
   interleaved bytes in imread's BGR order, converted with COLOR_BGR2GRAY whatever Camera.RGB says
   (src/line_detect/libs/binary_descriptor.cpp:490-495; OpenCV 3.2 RGB2Gray<uchar>,
   (B*1868 + G*9617 + R*4899 + 2^13) >> 14) -- not the tracker's mImGray when mbRGB = 1 (SURVEY
   Q20). The conversion is fused into the blur kernel's tile load (no gray plane). channels = 1 is
   eao_lines_detect. pitch in bytes (>= width * channels). */
int eao_lines_detect_color(eao_lines* l, const uint8_t* img, int pitch, int channels, float min_length,
                           float* lines, int cap, int* n_out);
/* eao_lines_detect_color in two halves, so the caller's thread does other work (the frame's
   extraction, matching and eao_replay_frame_begin) while the line detection runs on the handle's
   stream: _start stages the frame and enqueues every kernel, then returns; _finish waits and
   writes min(count, cap of _start) lines, with eao_lines_detect_color's return codes. One frame
   at a time per handle: _start with lines not yet taken, or _finish without _start, is
   EAO_E_STATE. img may be reused as soon as _start returns. */
int eao_lines_detect_color_start(eao_lines* l, const uint8_t* img, int pitch, int channels, float min_length,
                                 int cap);
int eao_lines_detect_finish(eao_lines* l, float* lines, int* n_out);
int eao_lines_detect_color_batch_device(eao_lines* l, const uint8_t* d_img, int nframes, int pitch, int channels,
                                        float min_length, float* d_lines, int32_t* d_counts, int cap,
                                        void* stream);
/* maps of the last eao_lines_detect: blur u8, Sobel dx / dy i16, code u16 = thresholded
   (|dx| + |dy|) / 4 | 0x8000 when |dx| < |dy| (Horizontal); NULL skips an output */
int eao_lines_debug_maps(eao_lines* l, uint8_t* blur, int16_t* dx, int16_t* dy, uint16_t* code);

/* --- EAO association: replaces Object_2D / Object_Map math (src/Object.cc) -- */
typedef struct {
  int32_t verdict; /* 0: m<20, 1: pass, 2: fail -- NoParaDataAssociation return */
  int32_t m, n;
  float w[3];
  float r1, r2;
  float cnt_gt[3], cnt_lt[3], cnt_eq[3];
} eao_np_stats;

typedef struct eao_assoc eao_assoc;
int eao_assoc_create(int device, int max_points, eao_assoc** out);
int eao_assoc_destroy(eao_assoc* a);

/* Object_2D::NoParaDataAssociation (src/Object.cc:714-930) for a batch of
   (detection, object) pairs. Point sets are float3 arrays with validity
   flags (!isBad && !out_point); pair p uses frame set fs[p] and object set
   os[p] given as offsets/lengths into the concatenated arrays. */
int eao_np_test_batch(eao_assoc* a, int npairs, const float* frame_pts, const uint8_t* frame_valid,
                      const int32_t* frame_off, const int32_t* frame_len, const float* obj_pts,
                      const uint8_t* obj_valid, const int32_t* obj_off, const int32_t* obj_len,
                      eao_np_stats* out);

/* IsolationForest::Build(trees, seed, data, sample) + GetAnomalyScores
   (include/isolation_forest.h:448-530) as called by
   Object_Map::IsolationForestDeleteOutliers (src/Object.cc:1257-1270), for a
   batch of point clouds (cloud c = pts[off[c] .. off[c]+len[c])). */
int eao_iforest_scores_batch(eao_assoc* a, int nclouds, const float* pts, const int32_t* off,
                             const int32_t* len, uint32_t trees, uint32_t seed,
                             const uint32_t* sample_size, double* scores);
/* The isolation-forest erase decision score > th (IsolationForestDeleteOutliers, th = 0.6f or
   0.65f for class 62, src/Object.cc:1284-1300) as the engine takes it: with
   x = -E[h] / c(psi), score = pow(2, x) exceeds th exactly when x >= *x0, x0 being the
   smallest double for which the host libm's pow(2, x) > th (so a device pow that differs
   by an ulp cannot flip an erasure). Host-only; no device needed. */
int eao_iforest_erase_threshold(float th, double* x0);

/* Object_Map::ComputeProjectRectFrame (src/Object.cc:1558-1603) for a batch of
   clouds under one pose; rect[c*4] = x,y,w,h (cv::Rect). Empty cloud -> rect
   left untouched and ok[c] = 0. */
int eao_project_rects(eao_assoc* a, const eao_camera* cam, const float* Tcw, int nclouds,
                      const float* pts, const int32_t* off, const int32_t* len, int32_t* rect,
                      uint8_t* ok);

/* Deterministic association replay: the object section
   of Tracking::TrackWithMotionModel (src/Tracking.cc:1241-1696) with
   ObjectDataAssociation / DataAssociateUpdate / iForest on the GPU, and the
   LocalMapping object maintenance (src/LocalMapping.cc:772-882). */
typedef struct eao_replay eao_replay;
int eao_replay_create(eao_assoc* a, const char* flag, int img_w, int img_h, const float* K4,
                      eao_replay** out);
int eao_replay_destroy(eao_replay* r);
int eao_replay_frame(eao_replay* r, int frame_id, const float* Tcw, int n_boxes,
                     const int32_t* boxes, int n_pts, const int32_t* mp_ids, const float* mp_pos,
                     const float* kp_uv, const uint8_t* mp_bad, int32_t* det_out);
int eao_replay_local_mapping(eao_replay* r);
/* eao_replay_frame in two calls around the frame's line detection: _begin runs the frame
   (map points, frame statistics, data association, the forest launches, culling) without its
   lines; the caller then stages the frame's lines (eao_replay_lines, one set) and _end runs
   AssociateObjAndLines and SampleObjYaw (Tracking.cc:1286, 1650-1671: the lines' only
   readers) and writes det_out as eao_replay_frame would. Same results as eao_replay_frame with
   the lines staged before it. Between the two calls eao_replay_frame, _begin,
   eao_replay_local_mapping and eao_replay_run return EAO_E_STATE; _end without an open frame
   too. _end returns #objects or < 0. */
int eao_replay_frame_begin(eao_replay* r, int frame_id, const float* Tcw, int n_boxes, const int32_t* boxes,
                           int n_pts, const int32_t* mp_ids, const float* mp_pos, const float* kp_uv,
                           const uint8_t* mp_bad);
int eao_replay_frame_end(eao_replay* r, int32_t* det_out);
/* Frame line segments (Frame::all_lines_eigen rows x1, y1, x2, y2 from the line
   detector, src/Frame.cc:324-335) for the next n_frames frames replayed by
   eao_replay_frame / eao_replay_run, one set per frame in order. They feed
   Tracking::AssociateObjAndLines (src/Tracking.cc:2472-2527) and SampleObjYaw
   (src/Tracking.cc:2624-2871, flags other than None / iForest). Frames without a
   staged set have no lines. */
int eao_replay_lines(eao_replay* r, int n_frames, const int32_t* n_lines, const float* lines);
/* a recorded stream in one call: frame t is eao_replay_frame on the t-th
   slices of the packed arrays (boxes / points concatenated over frames),
   followed by eao_replay_local_mapping when keyframe[t]. det_out receives 4
   ints per box in the same concatenated order. Returns #objects or < 0. */
int eao_replay_run(eao_replay* r, int n_frames, const int32_t* frame_ids, const float* Tcw,
                   const int32_t* n_boxes, const int32_t* boxes, const int32_t* n_pts,
                   const int32_t* mp_ids, const float* mp_pos, const float* kp_uv,
                   const uint8_t* mp_bad, const uint8_t* keyframe, int32_t* det_out);
/* LocalMapping's map-point changes for the points the association holds, applied in place:
   LocalBundleAdjustment's SetWorldPos (src/Optimizer.cc LocalBundleAdjustment ->
   src/MapPoint.cc:73-77), MapPointCulling / KeyFrameCulling's SetBadFlag (src/MapPoint.cc:151-167)
   and SearchInNeighbors' Replace (src/MapPoint.cc:175-220; the object keeps the old, now bad,
   point: Replace moves no object membership, so a replaced point is passed as bad = 1).
   pos [n][3] = GetWorldPos(), bad [n] = isBad(); either may be NULL to leave that field. Ids the
   replay never saw are ignored. The object code re-reads these at every later read
   (Object_Map::ComputeMeanAndStandard, src/Object.cc:967-992, called by LocalMapping::UpdateObject,
   src/LocalMapping.cc:772-795; NP tests, projected rects, forests, duplicate checks). The shim
   calls it from LocalMapping after LocalBA / KeyFrameCulling and before eao_replay_local_mapping
   (src/LocalMapping.cc:70-90). */
int eao_replay_update_points(eao_replay* r, int n, const int32_t* ids, const float* pos, const uint8_t* bad);
/* the ids of the map points the objects hold (ascending, unique): min(count, cap) written,
   count returned -- the set whose state a LocalMapping shim snapshots for the call above */
int eao_replay_held_points(eao_replay* r, int32_t* ids, int cap);
/* eao_replay_run with each frame's map-point record (the trace of SURVEY appendix B extended by
   LocalMapping's point changes): after frame t, the next n_upd[t] entries of upd_ids / upd_pos /
   upd_bad are applied as eao_replay_update_points, then eao_replay_local_mapping when keyframe[t].
   n_upd NULL = no records (eao_replay_run). Every forest of the stream has completed on return. */
int eao_replay_run_updates(eao_replay* r, int n_frames, const int32_t* frame_ids, const float* Tcw,
                           const int32_t* n_boxes, const int32_t* boxes, const int32_t* n_pts,
                           const int32_t* mp_ids, const float* mp_pos, const float* kp_uv,
                           const uint8_t* mp_bad, const uint8_t* keyframe, const int32_t* n_upd,
                           const int32_t* upd_ids, const float* upd_pos, const uint8_t* upd_bad,
                           int32_t* det_out);
/* Threading: every eao_replay_* call holds the handle's lock, so the Tracking thread
   (eao_replay_frame) and the LocalMapping thread (eao_replay_update_points,
   eao_replay_local_mapping) may share one handle; the replayed order is the order in which the
   calls take the lock. eao_replay_destroy takes no lock: the caller joins every other thread
   that uses the handle before destroying it.
   A stream call that fails part-way returns < 0 and drops the next frame's look-ahead state;
   a later eao_replay_frame / eao_replay_run continues from the last completed frame. */
int eao_replay_num_objects(eao_replay* r);
/* ints[8]: id, class, bad, #frames, #points, last add, #co-association votes, #co-views;
   floats[20]: center[3], sigma[3], sigma of frame centers[3], cuboid lenth/width/height,
   R_max, centre spread, projected rect x / w, rotY, #yaw measurements, mfErrorParallel,
   mfErroeYaw */
int eao_replay_object(eao_replay* r, int i, int32_t* ints, float* floats);
int eao_replay_object_points(eao_replay* r, int i, int32_t* ids, int cap);

/* Object-sharded association (Config C; replaces nothing in the
   reference, which is single-threaded here -- the sharded replay returns the
   same ids as eao_replay_frame). Every rank replays the same stream; the GPU
   work of object o (its NP pairs, projected rect, isolation forest) runs on
   rank o.id % world and the result records are all-gathered. Call before the
   first frame.
   eao_replay_shard_rccl: RCCL communicator (one device per rank, xGMI);
     unique_id = 128 bytes from eao_rccl_unique_id on one rank, broadcast. The
     records stay in device memory: the kernels write them, ncclAllGather reads
     them there behind a GPU-side event wait, and only the gathered records come
     back (one copy per exchange). World 1 is allowed and runs the whole exchange
     path on one device.
   eao_replay_shard_callback: the all-gather is the caller's (e.g. gloo), on host
     buffers; world 1 disables sharding. */
typedef int (*eao_allgather_fn)(void* ctx, const void* send, void* recv, size_t bytes_per_rank);
int eao_rccl_unique_id(uint8_t* out128);
/* One-rank self-test of the RCCL exchanger of eao_replay_shard_rccl: a world-1 communicator,
   device-to-device all-gathers of a kernel-written pattern of `bytes` and bytes + 4097
   (buffer regrowth), results compared. 0 = ok. */
int eao_rccl_selftest(int device, int bytes);
int eao_replay_shard_rccl(eao_replay* r, int rank, int world, const uint8_t* unique_id128);
int eao_replay_shard_callback(eao_replay* r, int rank, int world, eao_allgather_fn fn, void* ctx);
/* [0] exchanges, [1] bytes per rank, [2] us spent in the exchange */
int eao_replay_shard_stats(eao_replay* r, double* out3);
/* Self-test of the association's HSA launch lanes on `device` (no reference counterpart): completion
   markers held across many reuses of their signal slot, barrier packets on reused slots (held and
   committed), and runs of held packets meeting the ring end. 0 = ok (out1[0] = packets written);
   EAO_E_NODEVICE without a gfx950 device; else the failing step in eao_last_error(). */
int eao_lane_selftest(int device, int* out1);

/* development instrumentation: s_memtime stamps of the last isolation-forest
   tree launch (workgroup (0,0)), 32 entries: [0..7] phase boundaries, [10] node count,
   [12..29] sub-step cycle sums of EAO_IF_PROF builds. */
int eao_debug_iforest_stamps(uint64_t* out32);
/* wall-clock profile of a replay (us): [0] frame total, [1] local mapping,
   [2]/[3] iForest launches / time, [4]/[5] NP launches / time,
   [6]/[7] rect launches / time, [8] frames, [12..15] frame sections. */
int eao_replay_profile(eao_replay* r, double* out24);
/* The same wall-clock profile, up to n (<= 60) slots; returns the number copied. */
int eao_replay_profile_n(eao_replay* r, double* out, int n);

/* ---- frame input stage (src/Tracking.cc:340-554) ---- */
/* Tracking::GrabImageMonocular's offline detections: the text of one
   data/yolo_txts/<timestamp>.txt parsed as the reference does (`istr >> int` per line,
   so the score "0.82" reads as 0 -- SURVEY Q1), then std::sort by score descending.
   out: cap rows of {class, x, y, w, h, score}; *n_out = rows in the file
   (EAO_E_CAPACITY when > cap). Tracking.cc:426-472. Host-only. */
int eao_yolo_parse(const char* text, size_t len, int32_t* out, int cap, int* n_out);
/* The ground-truth pose lookup of every frame (Tracking.cc:506-554): gt = m rows of
   data/groundtruth.txt {t, tx, ty, tz, qx, qy, qz, qw}; for each timestamp the first row
   whose std::to_string(t) minus its last 4 characters equals the frame's; idx_out = row
   or -1; Twc_out (optional, n x 16 row-major float) = g2o::SE3Quat(row) as
   Converter::toCvMat gives it, zeros when no row matches. Host-only. */
int eao_gt_lookup(const double* gt, int m, const double* ts, int n, int32_t* idx_out, float* Twc_out);
/* cv::undistort(im, out, K, DistCoef) with an all-zero distortion model (TUM3.yaml:13-16,
   Tracking.cc:366-369): an exact per-pixel copy (the rectify map is the identity up to
   rounding that remap's fixed point absorbs); EAO_E_ARG for non-zero coefficients.
   src / dst host or device memory, copied on `stream` (NULL: the null stream). */
int eao_undistort_zero(const float* dist, int ndist, const uint8_t* src, int w, int h, int spitch, uint8_t* dst,
                       int dpitch, void* stream);

/* --- pose-only optimisation: replaces Optimizer::PoseOptimization (src/Optimizer.cc:243-457),
   monocular edges (mvuRight < 0), called at src/Tracking.cc:1106,1699,1741 --- */
typedef struct eao_pose eao_pose;
int eao_pose_create(int device, int max_kps, int max_batch, eao_pose** out);
int eao_pose_destroy(eao_pose* p);
/* one frame, host buffers: Tcw_in = pFrame->mTcw (4x4 row-major float); kps_un = mvKeysUn;
   has_mp[i] = mvpMapPoints[i] != NULL; mp_pos[3i..] = its GetWorldPos(); inv_level_sigma2 =
   mvInvLevelSigma2 (nlevels <= 32). Writes Tcw_out (SetPose), outlier[i] (mvbOutlier) where
   has_mp[i], and *n_inliers = the function's return value (0 with Tcw_out = Tcw_in when fewer
   than 3 correspondences, Optimizer.cc:370-371). */
int eao_pose_optimization(eao_pose* p, const eao_camera* cam, const float* Tcw_in, int n,
                          const eao_keypoint* kps_un, const uint8_t* has_mp, const float* mp_pos,
                          const float* inv_level_sigma2, int nlevels, float* Tcw_out, uint8_t* outlier,
                          int32_t* n_inliers);
/* batched, HBM-resident: frame f reads d_Tcw_in[f][16], d_counts[f] keypoints of
   d_kps_un / d_has_mp / d_mp_pos ([nframes][cap], positions [nframes][cap][3]) and writes
   d_Tcw_out[f][16], d_outlier[f][cap] (has_mp entries), d_n_inliers[f]; asynchronous on
   `stream` (the handle's stream when NULL). cap <= 8192. */
int eao_pose_optimization_batch_device(eao_pose* p, const eao_camera* cam, int nframes, int cap,
                                       const float* d_Tcw_in, const int32_t* d_counts,
                                       const eao_keypoint* d_kps_un, const uint8_t* d_has_mp,
                                       const float* d_mp_pos, const float* inv_level_sigma2, int nlevels,
                                       float* d_Tcw_out, uint8_t* d_outlier, int32_t* d_n_inliers,
                                       void* stream);

/* --- bag of words: Frame::ComputeBoW (src/Frame.cc:516-523 -> DBoW2
   TemplatedVocabulary::transform(desc, BowVector, FeatureVector, 4), TemplatedVocabulary.h:1139-1271;
   the ORB vocabulary's TF_IDF weighting + L1 norm) and ORBmatcher::SearchByBoW(KeyFrame*, Frame&,
   vector<MapPoint*>&) (src/ORBmatcher.cc:159-288), called at src/Tracking.cc (TrackReferenceKeyFrame,
   Relocalization) --- */
typedef struct eao_vocab eao_vocab;
/* the vocabulary as loadFromTextFile leaves it: node descriptors [n_nodes][32], parent[i] in
   [0, i) (root 0: parent -1), word_id[i] (-1: inner node), weight[i] (idf; 0 = stopped), depth L.
   n_nodes may be 0 (an empty vocabulary: transforms give empty vectors; searches still work).
   max_kps <= 4096 features per frame, max_batch frames per batched call. */
int eao_vocab_create(int device, int n_nodes, const uint8_t* node_desc, const int32_t* parent,
                     const int32_t* word_id, const double* weight, int L, int max_kps, int max_batch,
                     eao_vocab** out);
int eao_vocab_destroy(eao_vocab* v);
/* transform of one frame's n descriptors: BowVector as (word_ids ascending, word_weights) x
   *n_words; FeatureVector as CSR: node_ids ascending x *n_nodes, node_start [*n_nodes + 1],
   node_feats (feature indices, ascending within a node). Arrays hold >= n (+1) entries. */
int eao_bow_transform(eao_vocab* v, int n, const uint8_t* desc, int levelsup, int32_t* word_ids,
                      double* word_weights, int32_t* n_words, int32_t* node_ids, int32_t* node_start,
                      int32_t* node_feats, int32_t* n_nodes);
/* batched, HBM-resident: frame f reads d_counts[f] descriptors of d_desc [nframes][cap][32] and
   writes [nframes][cap] word ids / weights / node ids / node features, node starts
   [nframes][cap + 1] and the counts; asynchronous on `stream`. */
int eao_bow_transform_batch_device(eao_vocab* v, int nframes, int cap, const int32_t* d_counts,
                                   const uint8_t* d_desc, int levelsup, int32_t* d_word_ids,
                                   double* d_word_weights, int32_t* d_n_words, int32_t* d_node_ids,
                                   int32_t* d_node_start, int32_t* d_node_feats, int32_t* d_n_nodes,
                                   void* stream);
/* SearchByBoW(pKF, F, vpMapPointMatches): kf_mp_valid[i] = vpMapPointsKF[i] && !isBad(); the
   FeatureVectors as eao_bow_transform returns them. f_match[iF] = the keyframe feature whose map
   point F's feature iF matched (-1: none). Returns nmatches (>= 0) or an EAO_E_* error. */
int eao_search_by_bow(eao_vocab* v, float nnratio, int check_ori, int n_kf, const eao_keypoint* kf_kps,
                      const uint8_t* kf_desc, const uint8_t* kf_mp_valid, int kf_nn,
                      const int32_t* kf_node_ids, const int32_t* kf_node_start,
                      const int32_t* kf_node_feats, int n_f, const eao_keypoint* f_kps,
                      const uint8_t* f_desc, int f_nn, const int32_t* f_node_ids,
                      const int32_t* f_node_start, const int32_t* f_node_feats, int32_t* f_match);
/* batched, HBM-resident: search s pairs keyframe slot s with frame slot s ([nsearch][cap]
   keypoints / descriptors / valid flags / node ids / node features, [nsearch][cap + 1] node starts,
   per-search node counts d_kf_nn / d_f_nn and frame feature counts d_n_f); writes
   d_f_match [nsearch][cap] and d_nmatches [nsearch] (EAO_E_CAPACITY for a search in which a
   vocabulary node holds more than 1024 frame features). nsearch <= max_batch. Preconditions the
   device path does not check (eao_search_by_bow checks them on the host): node ids ascending,
   node starts non-decreasing from 0, every listed feature index in [0, count) of its side. */
int eao_search_by_bow_batch_device(eao_vocab* v, float nnratio, int check_ori, int nsearch, int cap,
                                   const eao_keypoint* d_kf_kps, const uint8_t* d_kf_desc,
                                   const uint8_t* d_kf_mp_valid, const int32_t* d_kf_nn,
                                   const int32_t* d_kf_node_ids, const int32_t* d_kf_node_start,
                                   const int32_t* d_kf_node_feats, const int32_t* d_n_f,
                                   const eao_keypoint* d_f_kps, const uint8_t* d_f_desc,
                                   const int32_t* d_f_nn, const int32_t* d_f_node_ids,
                                   const int32_t* d_f_node_start, const int32_t* d_f_node_feats,
                                   int32_t* d_f_match, int32_t* d_nmatches, void* stream);

/* ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12)
   (src/ORBmatcher.cc:522-655), called by LoopClosing::ComputeSim3 (src/LoopClosing.cc:265). Both sides as
   eao_search_by_bow's keyframe side: valid1 / valid2[i] = GetMapPointMatches()[i] && !isBad() (the second
   side's map points are checked too, :576-580), the FeatureVectors as eao_bow_transform returns them.
   match12[i1] = the KF2 feature whose map point KF1 feature i1 matched (-1: none) -- vpMatches12[i1] is that
   feature's map point. The distance bar is strict (bestDist1 < TH_LOW), the KF2 features are taken first-wins
   (vbMatched2), the rotation check histograms idx1. Returns nmatches (>= 0) or an EAO_E_* error. */
int eao_search_by_bow_kf(eao_vocab* v, float nnratio, int check_ori, int n1, const eao_keypoint* kps1,
                         const uint8_t* desc1, const uint8_t* valid1, int nn1, const int32_t* node_ids1,
                         const int32_t* node_start1, const int32_t* node_feats1, int n2, const eao_keypoint* kps2,
                         const uint8_t* desc2, const uint8_t* valid2, int nn2, const int32_t* node_ids2,
                         const int32_t* node_start2, const int32_t* node_feats2, int32_t* match12);
/* batched, HBM-resident: search s pairs KF1 slot s with KF2 slot s ([nsearch][cap] keypoints / descriptors /
   valid flags / node ids / node features, [nsearch][cap + 1] node starts, node counts d_nn1 / d_nn2, KF1 feature
   counts d_n1); writes d_match12 [nsearch][cap] and d_nmatches [nsearch] (EAO_E_CAPACITY for a search in which
   a vocabulary node holds more than 1024 KF2 features). nsearch <= max_batch; the FeatureVector
   preconditions of eao_search_by_bow_batch_device. */
int eao_search_by_bow_kf_batch_device(eao_vocab* v, float nnratio, int check_ori, int nsearch, int cap,
                                      const int32_t* d_n1, const eao_keypoint* d_kps1, const uint8_t* d_desc1,
                                      const uint8_t* d_valid1, const int32_t* d_nn1, const int32_t* d_node_ids1,
                                      const int32_t* d_node_start1, const int32_t* d_node_feats1,
                                      const eao_keypoint* d_kps2, const uint8_t* d_desc2, const uint8_t* d_valid2,
                                      const int32_t* d_nn2, const int32_t* d_node_ids2,
                                      const int32_t* d_node_start2, const int32_t* d_node_feats2,
                                      int32_t* d_match12, int32_t* d_nmatches, void* stream);

#ifdef __cplusplus
}
#endif
#endif
