/*
 * mage_hot.h — C-ABI of the MI355X-native MAGE-SLAM hot path.
 *
 * This is the drop-in boundary described in SURVEY.md §8(b).  Every entry point takes
 * plain pointers and sizes (no torch, OpenCV, Eigen or g2o types) and replaces one
 * reference interface, cited per function.  Reference paths are relative to the
 * marwie/mageslam tree; `Core/.../Source` = `Core/MAGESLAM/Source`.
 *
 * Status codes replace the reference's CV_Assert / assert failures; the C++ facades
 * (include/mage/mage.hpp) turn them back into exceptions so callers keep the reference
 * behaviour.
 */
#ifndef MAGE_HOT_H
#define MAGE_HOT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum mage_status {
    MAGE_OK = 0,
    MAGE_EINVAL = 1,        /* bad argument (reference: CV_Assert / assert) */
    MAGE_EDEVICE = 2,       /* HIP runtime error or no usable gfx950 device */
    MAGE_ENOMEM = 3,        /* device allocation failed */
    MAGE_EUNSUPPORTED = 4,  /* valid reference input this build does not handle yet */
    MAGE_ECAPACITY = 5      /* output capacity too small (outputs are truncated) */
} mage_status;

/* Layout-identical to cv::KeyPoint {Point2f pt; float size, angle, response; int octave, class_id}
 * as stored in ImageData (Core/.../Source/Image/ImageData.h:186-205). 28 bytes. */
typedef struct mage_keypoint {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} mage_keypoint;

/* Layout-identical to cv::DMatch {int queryIdx, trainIdx, imgIdx; float distance}. 16 bytes. */
typedef struct mage_dmatch {
    int32_t query_idx, train_idx, img_idx;
    float distance;
} mage_dmatch;

/* The 14 constructor scalars of OrbDetector (Core/.../Source/Image/OpenCVModified.h:68-82),
 * same order and meaning; defaults in FeatureExtractorSettings (MageSettings.h:151-167). */
typedef struct mage_orb_settings {
    uint32_t gaussian_kernel_size; /* 7 */
    uint32_t nfeatures;            /* 440 (2000 in the 720p benchmark) */
    float scale_factor;            /* 1.5 */
    uint32_t nlevels;              /* 1 */
    uint32_t patch_size;           /* 15 */
    uint32_t fast_threshold;       /* 4 */
    int32_t use_orientation;       /* 0 */
    float feature_factor;          /* 1.5 (ANMS) */
    float feature_strength;        /* 0.9 (ANMS) */
    int32_t strong_response;       /* 20 (ANMS) */
    float min_robust_factor;       /* 1.1 */
    float max_robust_factor;       /* 2.0 */
    int32_t num_cells_x;           /* 32 */
    int32_t num_cells_y;           /* 32 */
} mage_orb_settings;

/* Pyramid levels supported (nlevels in 1..MAGE_MAX_LEVELS). */
#define MAGE_MAX_LEVELS 8

typedef void* mage_stream; /* a hipStream_t; NULL = the default stream */

/* ------------------------------------------------------------------------------------------ */
/* Library                                                                                      */
/* ------------------------------------------------------------------------------------------ */

/* Version string and the gfx target the device code was compiled for ("gfx950"). */
const char* mage_version(void);
/* Last error message of the calling thread (empty string if none). */
const char* mage_last_error(void);
/* Frees the library's idle cached blocks (device, page-locked and mapped host memory retired by
 * destroyed per-task objects such as mage_ba) on `device` (-1: every device); returns the bytes
 * freed.  The cache keeps at most MAGE_POOL_CAP_MB (default 512) MB of idle device memory, a
 * quarter of that page-locked and a sixteenth mapped, frees blocks no request could use over 256
 * requests, and is trimmed automatically when an allocation fails.  No reference counterpart
 * (the reference allocates per task through new / cv::Mat). */
uint64_t mage_pool_trim(int32_t device);

/* Per-kernel timing: when enabled, every launch is bracketed by HIP events recorded on the
 * stream it is launched on.  The report is one line per kernel: "<name> <launches> <total_ms>". */
void mage_profile_enable(int32_t enable);
/* Time only the launches whose kernel tag starts with tag_prefix (null or "": all of them). */
void mage_profile_filter(const char* tag_prefix);
void mage_profile_reset(void);
const char* mage_profile_report(void);

/* ------------------------------------------------------------------------------------------ */
/* ORB extraction — replaces OrbDetector (Core/.../Source/Image/OpenCVModified.h:64-173)        */
/* ------------------------------------------------------------------------------------------ */

typedef struct mage_orb mage_orb;

/* OrbDetector::OrbDetector (OpenCVModified.cpp:362-393).  Also binds the HIP device. */
mage_status mage_orb_create(const mage_orb_settings* settings, int device, mage_orb** out);
mage_status mage_orb_destroy(mage_orb* orb);

/* OrbDetector::DetectAndCompute (OpenCVModified.cpp:771-886) on one 8-bit gray frame in host
 * memory; synchronous.  Writes up to `cap` keypoints (the ImageData capacity,
 * ImageData.h:65-70 truncates silently) and cap*32 descriptor bytes; *n = count.
 * Keypoint order is the canonical order of DESIGN.md §ORB (ANMS rank, else raster). */
mage_status mage_orb_detect_and_compute(mage_orb* orb, const uint8_t* img, int32_t width,
                                        int32_t height, int32_t stride, mage_keypoint* kp,
                                        uint8_t* desc, uint32_t cap, uint32_t* n);

/* Batched, device-resident form: `batch` frames at d_frames + f*frame_pitch (device memory),
 * outputs at d_kp + f*cap, d_desc + f*cap*32, d_n[f].  Asynchronous on `stream`. */
mage_status mage_orb_detect_and_compute_batch_device(mage_orb* orb, const uint8_t* d_frames,
                                                     uint32_t batch, int32_t width,
                                                     int32_t height, int32_t stride,
                                                     int64_t frame_pitch, mage_keypoint* d_kp,
                                                     uint8_t* d_desc, uint32_t cap,
                                                     uint32_t* d_n, mage_stream stream);

/* Sticky device-side status of the batched path (capacity overflow etc.): synchronises
 * `stream` and returns MAGE_OK, MAGE_ECAPACITY or MAGE_EUNSUPPORTED; reset clears it. */
mage_status mage_orb_status(mage_orb* orb, mage_stream stream);
mage_status mage_orb_reset_status(mage_orb* orb, mage_stream stream);

/* Candidate gate of the FAST pass (no reference counterpart; a speed-only state, DESIGN.md §2
 * ORB): each batch scores exactly only the pixels that can reach a gate G derived from the
 * detector's previous batch and re-runs the exact path for frames whose retain bound lies below
 * G, so outputs never depend on it.  set: the gate of the next batch on `level` (0 = none;
 * tests and tuning).  stats: the gate the last batch used, the gate the next batch will use and
 * how many frames of the last batch took the exact path again.  Both synchronise `stream`. */
mage_status mage_orb_set_fast_gate(mage_orb* orb, uint32_t level, int32_t gate, mage_stream stream);
mage_status mage_orb_fast_gate_stats(mage_orb* orb, uint32_t level, int32_t* last_gate,
                                     int32_t* next_gate, uint32_t* last_redo, mage_stream stream);

/* Benchmark/test input generator: writes frames t0..t0+count-1 of the seeded
 * panning texture sequence, each width*height bytes at d_out + i*frame_pitch.  Identical to
 * mageslam_amd/synth.py frame(). */
mage_status mage_synth_frames_device(uint8_t* d_out, uint32_t count, int32_t width,
                                     int32_t height, int64_t frame_pitch, uint32_t t0,
                                     uint64_t seed, mage_stream stream);

/* Benchmark / test input for the tracking loop (BASELINE.json C4): `count` frames of a textured plane
 * Z = plane_z seen by a pinhole camera; d_cams holds per frame R (row-major, world -> camera) and
 * the camera centre C (12 doubles).  Texel (floor(X s) + off, floor(Y s) + off) of the panning
 * sequence's texture; identical to mageslam_amd/synth.py scene_frames(). */
mage_status mage_synth_scene_device(uint8_t* d_out, uint32_t count, int32_t width, int32_t height,
                                    int64_t frame_pitch, const double* d_cams, double fx, double fy, double cx,
                                    double cy, double plane_z, double texel_scale, int64_t texel_offset,
                                    uint64_t seed, mage_stream stream);

/* FAST-9/16 score map of FAST_t<16> with NMS disabled-equivalent view: score[y*W+x] =
 * cornerScore if (x,y) passes the segment test, else 0 (OpenCVModified.cpp:1225-1512,
 * 927-1071).  Host buffers, synchronous.  Used for the VERIFY_SIMD-style parity check. */
mage_status mage_orb_fast_score_map(const uint8_t* img, int32_t width, int32_t height,
                                    int32_t stride, int32_t threshold, uint8_t* score_map,
                                    int device);

/* Camera calibration as OrbFeatureDetector::Process receives it (Device/CameraCalibration.h):
 * the linear intrinsics of GetCameraMatrix() and the OpenCV-ordered distortion coefficients of
 * GetCVDistortionCoeffs() — K1 K2 P1 P2 K3 (Poly3k, ndist = 5) [K4 K5 K6] (Rational6k, ndist = 8);
 * ndist = 0 for DistortionType::None. */
typedef struct mage_calibration {
    float fx, fy, cx, cy;
    float dist[8];
    int32_t ndist;
} mage_calibration;

/* OrbFeatureDetector::UndistortKeypoints (OrbFeatureDetector.cpp:30-62): keypoint positions
 * through cv::undistortPoints(pts, distorted.K, distorted.dist, noArray(), undistorted.K),
 * in place.  Process() calls it only when the two calibrations differ.  Host buffers. */
mage_status mage_undistort_keypoints(const mage_calibration* distorted, const mage_calibration* undistorted,
                                     mage_keypoint* kp, uint32_t n, int device);

/* Batched device form: frame f's keypoints at d_kp + f*pitch (pitch in keypoints), d_n[f] of
 * them (e.g. the outputs of mage_orb_detect_and_compute_batch_device).  Asynchronous. */
mage_status mage_undistort_keypoints_batch_device(const mage_calibration* distorted,
                                                  const mage_calibration* undistorted, mage_keypoint* d_kp,
                                                  int64_t pitch, const uint32_t* d_n, uint32_t batch,
                                                  mage_stream stream);

/* Frame undistortion — ImagePreprocessor::UndistortImage (ImagePreprocessor.cpp:71-120).  Create
 * once per (calibration, size): CalculateUndistortedCalibration (fx, fy kept, principal point at
 * the image centre; written to *undistorted if not NULL) and cv::initUndistortRectifyMap(K, dist,
 * noArray(), K', size, CV_32FC1) on the device.  Each frame: cv::remap(INTER_LINEAR,
 * BORDER_CONSTANT 0) of a width x height 8-bit image.  ndist must be 0, 4, 5 or 8.
 * Frames arrive as GRAYSCALE8 or as the Y plane of NV12 (CreateGrayCVMat, Utils/cv.cpp:8-28): the
 * stride / pitch arguments read either layout in place. */
typedef struct mage_undistorter mage_undistorter;
mage_status mage_undistorter_create(const mage_calibration* distorted, int32_t width, int32_t height, int device,
                                    mage_undistorter** out, mage_calibration* undistorted);
mage_status mage_undistorter_destroy(mage_undistorter* u);
/* The CV_32FC1 maps (map1 = x, map2 = y), width*height floats each, for tests. */
mage_status mage_undistorter_get_maps(mage_undistorter* u, float* mapx, float* mapy);
/* Host buffers, synchronous. */
mage_status mage_undistort_image(mage_undistorter* u, const uint8_t* src, int32_t src_stride, uint8_t* dst,
                                 int32_t dst_stride);
/* Batched device form: frame f at d_src + f*src_pitch -> d_dst + f*dst_pitch.  Asynchronous. */
mage_status mage_undistort_image_batch_device(mage_undistorter* u, const uint8_t* d_src, int32_t src_stride,
                                              int64_t src_pitch, uint8_t* d_dst, int32_t dst_stride, int64_t dst_pitch,
                                              uint32_t batch, mage_stream stream);

/* cv::resize(src, dst, Size(dw, dh), 0, 0, INTER_LINEAR) for CV_8UC1 (OpenCV 3.4.0 fixed-point
 * path, the pyramid levels' resize of OpenCVModified.cpp:833), any scale.  Device buffers,
 * asynchronous on `stream`. */
mage_status mage_resize_linear_device(const uint8_t* d_src, int32_t sw, int32_t sh, int32_t src_stride, uint8_t* d_dst,
                                      int32_t dw, int32_t dh, int32_t dst_stride, mage_stream stream);

/* Stereo frame preparation — ImagePreprocessor::ScaleImageForCameraConfiguration
 * (Core/.../Source/Image/ImagePreprocessor.cpp:18-65).  A camera as the reference passes it: its
 * MAGESlam::CameraConfiguration (Extrinsics: mage::Matrix M11..M44 row-major; Size) and the
 * undistorted pinhole CameraCalibration of the same size (fx, fy, cx, cy). */
typedef struct mage_camera_config {
    float extrinsics[16];
    float fx, fy, cx, cy;
    uint32_t width, height;
} mage_camera_config;

/* The geometry: targetToSource = source.Extrinsics * inverse(target.Extrinsics) (cv::Matx44f, LU
 * inverse), the overlap crop of the source frame in the target frame at max_depth_meters
 * (CalculateOverlapCropSourceInTarget, MageUtil.cpp:13-58; crop_xywh = the cv::Rect), *ok = 0 when
 * it lies entirely offscreen (IsEntirelyOffscreen, Utils/cv.h:405-418; the reference returns
 * false), else scaleSourceToTarget and the prepared camera: size (int)(size * scale) and
 * GetScaledIntrinsics (CameraCalibration.cpp:150-157) when scale != 1, the source otherwise.
 * Host only. */
mage_status mage_scale_for_camera_configuration(const mage_camera_config* source, const mage_camera_config* target,
                                                float max_depth_meters, int32_t crop_xywh[4], float* scale,
                                                mage_camera_config* prepared, int32_t* ok);

/* The whole call on a device image: the geometry above, then the source->width x source->height
 * image at d_src (src_stride) resized with INTER_LINEAR into d_dst (dst_stride; prepared->height
 * rows of prepared->width bytes; dst_capacity bytes available), or copied when scale == 1.
 * Nothing is written when *ok = 0.  Asynchronous on `stream`. */
mage_status mage_scale_image_for_camera_configuration_device(const mage_camera_config* source,
                                                             const mage_camera_config* target, float max_depth_meters,
                                                             const uint8_t* d_src, int32_t src_stride, uint8_t* d_dst,
                                                             int32_t dst_stride, int64_t dst_capacity,
                                                             mage_camera_config* prepared, float* scale, int32_t* ok,
                                                             mage_stream stream);

/* ------------------------------------------------------------------------------------------ */
/* Hamming matching — replaces FeatureMatcher (Core/.../Source/Tracking/FeatureMatcher.h)        */
/* ------------------------------------------------------------------------------------------ */

/* GetDescriptorDistance (FeatureMatcher.cpp:453-504): popcount(a ^ b) over 32 bytes. */
int32_t mage_hamming_distance(const uint8_t* a32, const uint8_t* b32);

/* Match (FeatureMatcher.cpp:61-190): masked two-way brute force with the ratio-delta test.
 * Masks may be NULL (= all true).  Host buffers, synchronous.  Output in ascending A index. */
mage_status mage_hamming_match(const uint8_t* desc_a, uint32_t n_a, const uint8_t* mask_a,
                               const uint8_t* desc_b, uint32_t n_b, const uint8_t* mask_b,
                               int32_t max_distance, int32_t min_difference, mage_dmatch* out,
                               uint32_t cap, uint32_t* n);

/* Batched device form: pair p matches A = d_desc_a + p*a_pitch (n_a[p] rows) against
 * B = d_desc_b + p*b_pitch (n_b[p] rows); no masks.  Results per pair at d_out + p*cap,
 * count in d_n[p].  d_n_a / d_n_b are device arrays.  Asynchronous on `stream`. */
mage_status mage_hamming_match_batch_device(const uint8_t* d_desc_a, int64_t a_pitch,
                                            const uint32_t* d_n_a, const uint8_t* d_desc_b,
                                            int64_t b_pitch, const uint32_t* d_n_b,
                                            uint32_t pairs, int32_t max_distance,
                                            int32_t min_difference, mage_dmatch* d_out,
                                            uint32_t cap, uint32_t* d_n, mage_stream stream);

/* RadiusMatch (FeatureMatcher.cpp:294-378, per query :386-446) against the target set's
 * KeypointSpatialIndex (KeypointSpatialIndex.cpp:46-106, replaced by an on-device band index):
 * a query matches targets with |x - qx| <= radius, |y - qy| <= radius and the same octave; best /
 * "second best" as the reference's loop visits candidates in ascending target index; accepted
 * when second - best > min_difference; then only matches whose distance is the unique minimum
 * among the matches to their target survive.  query_pos (n_query x 2 floats) overrides the query
 * positions (queryKeypointPositionOverrides); masks and query_pos may be NULL.  At most 4096
 * targets.  Host buffers, synchronous; output in query order (train_idx = target index). */
mage_status mage_radius_match(const mage_keypoint* query_kp, const float* query_pos,
                              const uint8_t* query_mask, const uint8_t* query_desc, uint32_t n_query,
                              const mage_keypoint* target_kp, const uint8_t* target_mask,
                              const uint8_t* target_desc, uint32_t n_target, float radius,
                              int32_t max_distance, int32_t min_difference, mage_dmatch* out,
                              uint32_t cap, uint32_t* n);

/* TrackLocalMap's per-map-point matching (TrackLocalMap.cpp:175-256: ProjectMapPointIntoCurrentFrame
 * -> MatchMapPointToCurrentFrame -> the single-query RadiusMatch of FeatureMatcher.cpp:386-446) over
 * projected map points in order: point i searches the frame keypoints in its box (|x - qx| <=
 * radius, |y - qy| <= radius, same octave) that are still unassociated (mask[t] != 0), keeps the best
 * Hamming distance with the reference's "second = previous best" rule (candidates in ascending
 * keypoint order) and, when best <= max_distance and second - best > min_difference, associates
 * keypoint t: result[i] = t and mask[t] = 0 for every later point.  query_hide[i] >= 0 is the
 * keypoint a pose-estimation outlier point was matched to, hidden from its own search (:192-229);
 * NULL = none.  result[i] = -1 when no match.  Host buffers, synchronous; n_target <= 4096. */
mage_status mage_local_map_match(const float* query_pos, const int32_t* query_octave, const uint8_t* query_desc,
                                 const int32_t* query_hide, uint32_t n_query, const mage_keypoint* target_kp,
                                 const uint8_t* target_desc, uint32_t n_target, uint8_t* mask, float radius,
                                 int32_t max_distance, int32_t min_difference, int32_t* result, int device);

/* Batched device form, one (query set, target set) pair per workgroup: pair p reads
 * query_pitch / target_pitch entries further on (keypoints, positions, 32-byte descriptors),
 * counts from d_n_query[p] / d_n_target[p]; no masks.  d_scratch: pairs x query_pitch int32.
 * Results at d_out + p*cap, count in d_n[p]; bit 0 of *d_status is set when a target set exceeds
 * 4096 (that pair reports 0 matches).  Asynchronous on `stream`. */
mage_status mage_radius_match_batch_device(const mage_keypoint* d_query_kp, const float* d_query_pos,
                                           const uint8_t* d_query_desc, int64_t query_pitch,
                                           const uint32_t* d_n_query, const mage_keypoint* d_target_kp,
                                           const uint8_t* d_target_desc, int64_t target_pitch,
                                           const uint32_t* d_n_target, uint32_t pairs, float radius,
                                           int32_t max_distance, int32_t min_difference,
                                           int32_t* d_scratch, mage_dmatch* d_out, uint32_t cap,
                                           uint32_t* d_n, uint32_t* d_status, mage_stream stream);

/* ------------------------------------------------------------------------------------------ */
/* Vocabulary tree + IndexedMatch — replaces OnlineBow::FindLeafNode / QueryFeatures and          */
/* IndexedMatch (Core/.../Source/BoW/OnlineBow.cpp, Tracking/FeatureMatcher.cpp:192-292)          */
/* ------------------------------------------------------------------------------------------ */

typedef struct mage_bow mage_bow;

/* The OnlineBow tree as CreateTree / Kmean build it (OnlineBow.cpp:325-411): node i has the
 * 32-byte descriptor node_desc + 32 i and children children[child_start[i] .. child_start[i+1])
 * in childrenIDs order; node 0 is the root.  Children must have larger ids than their parent
 * (Kmean appends them after it) — MAGE_EINVAL otherwise. */
mage_status mage_bow_create(const uint8_t* node_desc, const uint32_t* child_start, const uint32_t* children,
                            uint32_t n_nodes, int device, mage_bow** out);
/* OnlineBow::CreateTree (Core/MAGESLAM/Source/BoW/OnlineBow.cpp:325-337) over n training
 * descriptors (host, 32 B each): hierarchical Kmean (:451-485) with InitializeTraining's
 * std::shuffle(mt19937{}) (:396-411, MSVC STL algorithm), IterateClusteringKmean (:587-614),
 * KmeanCenter (:551-585) and FindCluster (:631-638) — the clustering iterations run on the GPU,
 * every node of a tree level at once.  levels / branching / max_iter = BagOfWordsSettings
 * TrainingTreeLevels / TrainingTreeBranchingFactor / MaxTrainingIteration (MageSettings.h:230-232;
 * branching <= 16 here).  Node ids follow the reference's recursion.  SetNodeWeights (IDF) is host
 * bookkeeping over mage_bow_find_leaves (mageslam_amd/bow.py OnlineBow). */
mage_status mage_bow_train(const uint8_t* desc, uint32_t n, uint32_t levels, uint32_t branching, uint32_t max_iter,
                           int device, mage_bow** out);
/* The same tree built by OnlineBow::Kmedoid (OnlineBow.cpp:487-521, IterateClusteringKmedoid
 * :590-639) instead of Kmean: every node is the member of its group with the first smallest sum of
 * distances to the group (an empty group keeps its medoid; the reference reads past an empty
 * vector there). */
mage_status mage_bow_train_kmedoid(const uint8_t* desc, uint32_t n, uint32_t levels, uint32_t branching,
                                   uint32_t max_iter, int device, mage_bow** out);
/* The tree of `bow` (node_desc n x 32, child_start n + 1, children n - 1); MAGE_ECAPACITY with
 * *n_nodes set when cap_nodes is too small. */
mage_status mage_bow_get_tree(mage_bow* bow, uint8_t* node_desc, uint32_t* child_start, uint32_t* children,
                              uint32_t cap_nodes, uint32_t* n_nodes);
mage_status mage_bow_destroy(mage_bow* bow);

/* FindLeafNode (OnlineBow.cpp:289-311) of n descriptors: leaf[i] = node id.  Host buffers,
 * synchronous; _device: device buffers, asynchronous on `stream`. */
mage_status mage_bow_find_leaves(mage_bow* bow, const uint8_t* desc, uint32_t n, uint32_t* leaf);
mage_status mage_bow_find_leaves_device(mage_bow* bow, const uint8_t* d_desc, uint32_t n, uint32_t* d_leaf,
                                        mage_stream stream);

/* IndexedMatch (FeatureMatcher.cpp:192-292) with the BoW candidate lists (OnlineBowFeatureMatcher::
 * QueryFeatures / OnlineBow::QueryFeatures: the other image's features in the query's leaf, in
 * index order): forward TrackMatch best / second best, accepted when best < max_distance + 1 and
 * (second >= max_distance + 1 or second - best >= min_difference); kept when the reverse match
 * of B[j] over A's features of the same leaf returns A[i] with the same test.  Masks may be NULL
 * (all true).  At most 4096 features per side.  Host buffers, synchronous; output in A order,
 * DMatch(queryIdx = A index, trainIdx = B index, imgIdx = -1, distance). */
mage_status mage_indexed_match(mage_bow* bow, const uint8_t* desc_a, uint32_t n_a, const uint8_t* mask_a,
                               const uint8_t* desc_b, uint32_t n_b, const uint8_t* mask_b, int32_t max_distance,
                               int32_t min_difference, mage_dmatch* out, uint32_t cap, uint32_t* n);

/* Batched device form, one (A, B) pair per workgroup, leaves precomputed (e.g. by
 * mage_bow_find_leaves_device): pair p reads a_pitch / b_pitch entries further on (descriptors,
 * leaves, optional masks), counts d_n_a[p] / d_n_b[p].  Results at d_out + p*cap, count in d_n[p];
 * bit 0 of *d_status is set when a side exceeds 4096 (that pair reports 0).  Asynchronous. */
mage_status mage_indexed_match_batch_device(const uint8_t* d_desc_a, const uint32_t* d_leaf_a, const uint8_t* d_mask_a,
                                            int64_t a_pitch, const uint32_t* d_n_a, const uint8_t* d_desc_b,
                                            const uint32_t* d_leaf_b, const uint8_t* d_mask_b, int64_t b_pitch,
                                            const uint32_t* d_n_b, uint32_t pairs, int32_t max_distance,
                                            int32_t min_difference, mage_dmatch* d_out, uint32_t cap, uint32_t* d_n,
                                            uint32_t* d_status, mage_stream stream);

/* ------------------------------------------------------------------------------------------ */
/* Local bundle adjustment — replaces BundlerLib (Dependencies/BundlerLib/Include/BundlerLib.h) */
/* ------------------------------------------------------------------------------------------ */

typedef struct mage_ba mage_ba;

/* BundlerLib::BundlerLib(BundlerParameters{ArePointsFixed}) (BundlerLib.cpp:184-196). */
mage_status mage_ba_create(int32_t points_fixed, int device, mage_ba** out);
mage_status mage_ba_destroy(mage_ba* ba);

/* AllocateCameras + SetCameraPose for all cameras (BundlerLib.cpp:198-207, 261-278).
 * pos3: view-space position t (3 floats/camera); R9: rotation, Eigen column-major
 * (9 floats/camera); intr4: {cx, cy, fx, fy}; fixed: 0/1.  Only fx is used as the focal
 * length, as in the reference (CameraParameters(intr[2], (intr[0], intr[1]), 0)). */
mage_status mage_ba_set_cameras(mage_ba* ba, uint32_t n, const float* pos3, const float* r9,
                                const float* intr4, const uint8_t* fixed);
/* FixCameraPose (BundlerLib.cpp:280-283). */
mage_status mage_ba_fix_camera(mage_ba* ba, uint32_t idx, int32_t fixed);
/* AllocateMapPoints + SetMapPoint (BundlerLib.cpp:209-217, 285-292). */
mage_status mage_ba_set_points(mage_ba* ba, uint32_t n, const float* xyz);
/* AllocateObservations + SetObservation (BundlerLib.cpp:219-229, 294-309). */
mage_status mage_ba_set_observations(mage_ba* ba, uint32_t n, const float* uv,
                                     const uint32_t* cam, const uint32_t* pt,
                                     const float* info);
/* SetCurrentLambda / GetCurrentLambda (BundlerLib.cpp:354-362). */
mage_status mage_ba_set_lambda(mage_ba* ba, float lambda);
mage_status mage_ba_get_lambda(mage_ba* ba, float* lambda);
/* Tether constraints: Allocate*Constraints(n) + Set*Constraint(i, ...) for one kind
 * (BundlerLib.cpp:229-257, 311-350; called from BundleAdjust.cpp:155-189).  Replaces the set of
 * that kind; the others are kept.  params per tether:
 *   MAGE_TETHER_DISTANCE  (SetFixedDistanceConstraint)     1 float: distance
 *   MAGE_TETHER_ROTATION  (SetRelativeRotationConstraint)  4 floats: quaternion x, y, z, w
 *   MAGE_TETHER_TRANSFORM (SetRelativeTransformConstraint) 7 floats: position x, y, z, then
 *                                                          quaternion x, y, z, w
 * weight[i] is the constraint weight.  Camera indices must be < the camera count and distinct
 * (MAGE_EINVAL otherwise); set the cameras first. */
enum { MAGE_TETHER_DISTANCE = 0, MAGE_TETHER_ROTATION = 1, MAGE_TETHER_TRANSFORM = 2 };
mage_status mage_ba_set_tethers(mage_ba* ba, uint32_t kind, uint32_t n, const uint32_t* cam1,
                                const uint32_t* cam2, const float* params, const float* weight);

/* StepBundleAdjustment (BundlerLib.cpp:364-447): one LM iteration per entry of huber[],
 * stopping early if an iteration fails; then the outlier / cheirality pass.  Outlier
 * observation indices are appended in ascending order (g2o active-edge order) to
 * outliers[0..cap); *n_out = number reported.  *mean_sq = Σ‖e‖²/count over kept edges
 * (NaN if none, as the reference's 0/0). */
mage_status mage_ba_step(mage_ba* ba, const float* huber, uint32_t nsteps,
                         float max_error_square, uint32_t* outliers, uint32_t cap,
                         uint32_t* n_out, float* mean_sq);

/* GetPose / GetPoint (BundlerLib.cpp:457-471), all at once. */
mage_status mage_ba_get_poses(mage_ba* ba, float* pos3, float* r9);
mage_status mage_ba_get_points(mage_ba* ba, float* xyz);

/* The fp64 estimate itself: qt7 = {qx, qy, qz, qw, tx, ty, tz} per camera, xyz per point
 * (either may be NULL).  Used by the parity tests; the reference exposes only the float casts. */
mage_status mage_ba_get_state_f64(mage_ba* ba, double* qt7, double* xyz);

/* Instrumentation: counters since creation. */
typedef struct mage_ba_stats {
    uint64_t iterations;      /* LM solve() calls */
    uint64_t trials;          /* LM inner trials (linear solves) */
    uint64_t rejected_trials; /* trials that popped the state */
    double last_chi2;         /* robust chi2 after the last iteration */
    double lambda;            /* current LM lambda */
} mage_ba_stats;
mage_status mage_ba_get_stats(mage_ba* ba, mage_ba_stats* stats);

/* Batched pose-only BA: TrackLocalMap::OptimizeCameraPose (TrackLocalMap.cpp:421-501) for many
 * independent frames in one launch.  Problem k = a fresh BundlerLib with ArePointsFixed, camera 0 =
 * (pos3[k], r9[k] column-major, intr4[k] = {cx, cy, fx, fy}, not fixed), observations obs_start[k] ..
 * obs_start[k+1]-1 each on its own fixed map point (points3, uv, info = MapPointRefinementConfidence),
 * then StepBundleAdjustment(nsteps x huber, max_error_square).  Outputs per problem: GetPose(0)
 * (pos3_out, r9_out column-major), mean_sq (the post-pass mean, NaN if nothing kept), optionally
 * qt7_out (fp64 q xyzw + t) and stats {LM iterations, trials}; per observation outlier = 1 where
 * the post-pass rejects it (outlierIndices = the flagged indices, ascending).  Host buffers,
 * synchronous; _device: device buffers, asynchronous on `stream`. */
mage_status mage_ba_pose_batch(uint32_t problems, const float* pos3, const float* r9, const float* intr4,
                               const uint32_t* obs_start, const float* points3, const float* uv, const float* info,
                               uint32_t nsteps, float huber, float max_error_square, float* pos3_out, float* r9_out,
                               double* qt7_out, uint8_t* outlier, float* mean_sq, uint32_t* stats, int device);
mage_status mage_ba_pose_batch_device(uint32_t problems, const float* d_pos3, const float* d_r9, const float* d_intr4,
                                      const uint32_t* d_obs_start, const float* d_points3, const float* d_uv,
                                      const float* d_info, uint32_t nsteps, float huber, float max_error_square,
                                      float* d_pos3_out, float* d_r9_out, double* d_qt7_out, uint8_t* d_outlier,
                                      float* d_mean_sq, uint32_t* d_stats, mage_stream stream);

/* ---------------------------------------------------------------------------------------------
 * C4 tracking loop (native host code over mage_radius_match + mage_ba_pose_batch): per frame the
 * constant-velocity prediction, ProjectUndistorted of the reference keyframe's map points and
 * RadiusMatch at SearchRadius / WiderSearchRadius / ExtraWiderSearchRadius
 * (PoseEstimator::TryEstimatePoseFromKeyframe, Core/MAGESLAM/Source/Tracking/PoseEstimator.cpp:
 * 439-607), TrackLocalMap's two OptimizeCameraPose passes (TrackLocalMap.cpp:37-140) and the
 * keyframe decision of NewKeyFrameDecision.cpp:196.  A keyframe's map points are its keypoints
 * back-projected onto the plane Z = plane_z (the reference triangulates; outside the hot path).
 * Same specification, expression by expression, as mageslam_amd/tracking.py's `track`.
 * --------------------------------------------------------------------------------------------- */
typedef struct mage_track_settings {
    float search_radius, wider_search_radius, extra_wider_search_radius; /* 12, 24, 36 px */
    double small_match_ratio;                                            /* FeatureSmallMatchRatioThreshold */
    uint32_t min_matches;
    int32_t max_hamming, min_hamming_difference;                         /* 30, 1 */
    uint32_t initial_steps;                                              /* 3 */
    float initial_huber;                                                 /* 4 */
    double initial_max_error;                                            /* 6 (squared inside) */
    uint32_t final_steps;                                                /* 4 */
    float final_huber;                                                   /* 0.9 */
    double final_max_error;                                              /* 4.5 */
    /* FIXED (deprecated; kept for ABI layout): must equal MapPointRefinementConfidence(0) =
     * 1 - 1/1.5^2, else MAGE_EINVAL.  Observation information now follows each map point's own
     * refinement count (MappingMath.h:42-49); the field will be dropped at the next ABI bump. */
    float refinement_info;
    double keyframe_ratio;                                               /* 0.5 */
    uint32_t keyframe_min;                                               /* 25 */
    /* TrackLocalMap's local-map search between the two pose passes (TrackLocalMap.cpp:114-265,
     * TrackLocalMapSettings MageSettings.h:180-194); local_map_keyframes = 0 turns it off.  The
     * local map is the last local_map_keyframes keyframes, visited in ascending keyframe id. */
    uint32_t local_map_keyframes;                                        /* 4 (<= 8) */
    float match_search_radius;                                           /* MatchSearchRadius 8 */
    int32_t local_max_hamming, local_min_hamming_difference;             /* OrbMatcherSettings 30, 1 */
    float min_view_cos;         /* cosf(deg2rad(MinDegreesBetweenCurrentViewAndMapPointView = 60)) */
    float image_border;                                                  /* PatchSize / 2 = 7.5 */
    uint32_t min_tracked;                                                /* MinTrackedFeatureCount 20 */
    float scale_factor;                                                  /* pyramid ScaleFactor 1.5 */
    uint32_t num_levels;                                                 /* pyramid levels 1 */
    int32_t width, height;                                               /* image size */
    /* Local bundle adjustment after every new keyframe (MappingWorker.cpp:228-371; device loop
     * only, mage_track_sequence refuses it): over the local map's keyframes, the free ones and the
     * points they observe chosen as GetMapPointsAndDistantKeyframes does (ThreadSafeMap.cpp:
     * 888-957, see ba_free_keyframes), every alive association of those points; one
     * StepBundleAdjustment per keyframe at MaxOutlierError with the persisted lambda and
     * covisibility threshold (tracking.py local_bundle_adjust). */
    uint32_t local_ba;                                                   /* 0: off */
    float ba_huber, ba_huber_scale, ba_max_outlier_error;                /* 1.8, 0.95, 7.25 */
    uint32_t ba_steps_per_run;                                           /* NumStepsPerRun 1 */
    float ba_low_connectivity_scale;                                     /* 1.5 */
    uint32_t ba_upper_connections;                                       /* UpperConnectionsForBA 2000 */
    float min_lambda;                                                    /* MappingSettings::MinLambda 1e-3 */
    /* 0 (default): the new keyframe Ki and the keyframes sharing >= theta map points with it are
     * free, every other observer and the sequence's first keyframe fixed; theta starts at
     * covis_min_threshold, steps by covis_ba_step while the associations lie outside
     * [ba_lower_connections, ba_upper_connections] (covis_max_steps + 1 rounds) and persists
     * across windows.  N > 0: the newest N keyframes of the window free, the older ones fixed. */
    uint32_t ba_free_keyframes;
    uint32_t covis_min_threshold;                                        /* CovisMinThreshold 15 */
    uint32_t covis_ba_step;                                              /* CovisBaStepThreshold 15 */
    uint32_t ba_lower_connections;                                       /* LowerConnectionsForBA 1500 */
    uint32_t covis_max_steps;                                            /* MaxSteps 1 */
    /* New map points' depth x (1 + sigma g), g a seeded unit-variance variate per (keyframe frame,
     * keypoint) (tracking.py depth_noise_factor): a triangulated point's depth error instead of the
     * plane back-projection's exact depth.  0: exact. */
    float map_point_depth_noise;
} mage_track_settings;

/* Features of `frames` frames (host): keypoints kp[frame_start[f] .. frame_start[f+1]) and their
 * descriptors (32 B each); K = {fx, fy, cx, cy}; first_pose = R (row-major, world -> camera) and
 * t of frame 0 (its keyframe).  Outputs per frame: poses (R row-major + t, 12 doubles), the
 * RadiusMatch count, the inliers after both passes (0 when lost) and the keyframe flag. */
mage_status mage_track_sequence(const mage_keypoint* kp, const uint8_t* desc, const uint32_t* frame_start,
                                uint32_t frames, const double K[4], const double first_pose[12], double plane_z,
                                const mage_track_settings* settings, double* poses, uint32_t* matches,
                                uint32_t* inliers, uint8_t* keyframe, int device);

/* The same loop device-resident (csrc/track.hip): features in device memory as the batched
 * extraction leaves them — frame f's keypoints at d_kp + f*pitch (pitch <= 4096), descriptors at
 * d_desc + 32*f*pitch, count d_n[f]; every per-frame decision (fallback radii, lost frames,
 * keyframes) is taken on the device, the host enqueues all frames on `stream` and synchronises
 * once.  Outputs (host) as mage_track_sequence, identical to it. */
mage_status mage_track_sequence_device(const mage_keypoint* d_kp, const uint8_t* d_desc, uint32_t pitch,
                                       const uint32_t* d_n, uint32_t frames, const double K[4],
                                       const double first_pose[12], double plane_z,
                                       const mage_track_settings* settings, double* poses, uint32_t* matches,
                                       uint32_t* inliers, uint8_t* keyframe, uint32_t* ba_outliers,
                                       mage_stream stream);

#ifdef __cplusplus
}
#endif

#endif /* MAGE_HOT_H */
