/*
 * gtsfm_hip.h — C ABI of the MI355X-native GTSfM two-view front-end (libgtsfm_hip.so, gfx950).
 *
 * Every entry point takes plain pointers and sizes. Pointers named d_* are DEVICE pointers (HBM);
 * `stream` is a hipStream_t passed as void* (NULL = default stream). No entry point allocates,
 * synchronises or copies to the host: callers own every buffer and size workspaces with the
 * matching *_workspace_bytes() query, so a call can be captured into a hipGraph.
 * Return value: GTSFM_OK (0) or a negative GTSFM_ERR_* code. Degenerate DATA (too few matches,
 * no model) is never an error: it is reported per pair, as the reference reports a failure tuple.
 *
 * Reference interfaces replaced (file:line in alphonse-CHEN/gtsfm @ 2025-01-17):
 *   gtsfm_match_*           <- gtsfm/frontend/matcher/twoway_matcher.py:42-144 TwoWayMatcher.match
 *                              (cv.BFMatcher(NORM_L2).knnMatch(k=2) x 2 directions + ratio + mutual + sort)
 *   gtsfm_ransac_*          <- gtsfm/frontend/verifier/opencv_verifier_base.py:45-109 verify +
 *                              gtsfm/frontend/verifier/ransac.py:52-82 estimate_E +
 *                              gtsfm/utils/verification.py:52-94 recover_relative_pose_from_essential_matrix +
 *                              gtsfm/frontend/inlier_support_processor.py:39-95 run_inlier_support
 *   gtsfm_sift_*            <- gtsfm/frontend/detector_descriptor/sift.py:27-56 detect_and_describe
 *                              (cv.cvtColor RGB2GRAY + cv.SIFT_create().detectAndCompute + Keypoints.get_top_k)
 *   gtsfm_retrieval_*       <- gtsfm/retriever/netvlad_retriever.py:77-228 (similarity blocks + pairs_from_score_matrix)
 *   gtsfm_netvlad_*         <- gtsfm/frontend/global_descriptor/netvlad_global_descriptor.py:27-46 describe +
 *                              thirdparty/hloc/netvlad.py:28-71 (NetVLADLayer), :160-191 (NetVLAD.forward)
 */
#ifndef GTSFM_HIP_H_
#define GTSFM_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GTSFM_OK 0
#define GTSFM_ERR_ARG (-1)      /* invalid argument (shape, null pointer, unsupported mode) */
#define GTSFM_ERR_HIP (-2)      /* a HIP runtime call failed */
#define GTSFM_ERR_CAPACITY (-3) /* workspace too small */

/* ----------------------------------------------------------------------------------------------
 * Library
 * ---------------------------------------------------------------------------------------------- */
/* ABI version (major*100 + minor); a binding built against this header checks that the library
 * returns GTSFM_HIP_ABI_VERSION before binding anything else. */
#define GTSFM_HIP_ABI_VERSION 402
int gtsfm_hip_abi_version(void);
/* Name of the offload target the kernels were compiled for (e.g. "gfx950"). */
const char* gtsfm_hip_target(void);

/* ----------------------------------------------------------------------------------------------
 * Matcher: mutual nearest neighbour + Lowe ratio test over a batch of image pairs.
 *
 * Descriptors of all images live in one padded array d_desc[n_img][kmax][dim] float32 with
 * d_counts[n_img] valid rows per image. d_pairs[n_pairs][2] holds (i1, i2) image indices.
 * Output: d_out_idx[n_pairs][kmax][2] uint32 (i1 keypoint, i2 keypoint) and d_out_count[n_pairs];
 * rows 0..count-1 of each pair are ordered exactly like TwoWayMatcher.match's result
 * (ascending 1->2 distance, ties by i1 index). ratio < 0 disables the ratio test.
 *
 * mode GTSFM_MATCH_EXACT_F32: any float descriptors; distances are sum_k (a_k-b_k)^2 in float32,
 *      sequential k (bit-exact with the oracle; equals OpenCV for integer data or dim == 1).
 * mode GTSFM_MATCH_INT_F16:   integer-valued descriptors in [0, 1023] with squared norm < 2^19
 *      (every SIFT descriptor). One fp16 MFMA distance GEMM per pair with the norms and a 4-bit row code
 *      folded into extra K columns (every accumulator is d2 + code/16, exact in any summation order), fused
 *      row/column top-2. Exact integer arithmetic: bit-identical to EXACT_F32.
 *      kmax <= 8192, dim <= 139. (EXACT_F32: kmax <= 65535.)
 * mode GTSFM_MATCH_F16_RERANK: any float descriptors with dim <= 256 (e.g. SuperPoint's 256-D unit vectors).
 *      An fp16 MFMA distance GEMM shortlists 8 candidates per keypoint and side, an exact fp32 re-rank with
 *      EXACT_F32's arithmetic recomputes them, and a rounding-error certificate proves the shortlist holds the
 *      exact top 2; uncertified keypoints (and images with |value| > 60000 or non-finite values) are rescanned
 *      exactly. Bit-identical to EXACT_F32. dim > 256 runs the EXACT_F32 kernels. kmax <= 65535.
 * ---------------------------------------------------------------------------------------------- */
#define GTSFM_MATCH_EXACT_F32 0
#define GTSFM_MATCH_INT_F16 1
#define GTSFM_MATCH_F16_RERANK 2

size_t gtsfm_match_workspace_bytes(int n_img, int kmax, int dim, int n_pairs, int mode);

int gtsfm_match_batched(const float* d_desc, const int* d_counts, int n_img, int kmax, int dim,
                        const int* d_pairs, int n_pairs, double ratio, int mode, void* d_workspace,
                        size_t workspace_bytes, uint32_t* d_out_idx, int* d_out_count, void* stream);

/* gtsfm_match_batched with the INT_F16 distance GEMM's work laid out by the caller (no reference counterpart: the
 * reference matches one pair per call, twoway_matcher.py:42-144 via det_desc_correspondence_generator.py:60-75).
 * d_groups[n_groups][group_size] lists pair indices (-1 = empty slot); every pair must appear exactly once, and the
 * pairs of one group should share image i1 (the operand a workgroup keeps in registers: it is then read once per
 * group instead of once per pair; a group mixing i1 images is correct, only slower). group_size <=
 * gtsfm_match_max_group(kmax, dim). Group order sets which workgroups run side by side on an XCD: consecutive groups
 * that stream the same few i2 images share that XCD's L2. d_groups == NULL is gtsfm_match_batched. Other modes
 * ignore the groups. */
int gtsfm_match_batched_grouped(const float* d_desc, const int* d_counts, int n_img, int kmax, int dim,
                                const int* d_pairs, int n_pairs, const int* d_groups, int n_groups, int group_size,
                                double ratio, int mode, void* d_workspace, size_t workspace_bytes,
                                uint32_t* d_out_idx, int* d_out_count, void* stream);

/* Largest group_size gtsfm_match_batched_grouped accepts for this kmax / dim (its LDS holds the column state of every
 * pair of a group); 0 when INT_F16 does not support the shape. */
int gtsfm_match_max_group(int kmax, int dim);

/* Measurement hook (no reference counterpart): hipEvent_t handles recorded on the call's stream immediately before
 * and after the distance-GEMM kernel of every later GTSFM_MATCH_INT_F16 gtsfm_match_batched call, so a benchmark can
 * time that one kernel. NULL, NULL switches it off. Process-wide; not thread-safe. */
int gtsfm_match_set_kernel_events(void* hip_event_start, void* hip_event_stop);

/* Measurement hook (no reference counterpart): after a GTSFM_MATCH_F16_RERANK gtsfm_match_batched call (dim <= 256) has
 * completed on `stream`, the number of (keypoint, side) entries whose fp16 shortlist was not certified (and were
 * recomputed exactly), and optionally per pair and side (h_uncertified_per_side[side * n_pairs + p], side 0 = rows of
 * i1). A (pair, side) with at least 1/32 of its keypoints uncertified is recomputed whole by the exact tile kernel,
 * the rest one keypoint at a time. Same workspace and shape arguments as the call; blocks until the copies land. */
int gtsfm_match_rerank_stats(const void* d_workspace, size_t workspace_bytes, int n_img, int kmax, int dim,
                             int n_pairs, int* h_uncertified, int* h_uncertified_per_side, void* stream);

/* ----------------------------------------------------------------------------------------------
 * Verifier: essential-matrix RANSAC over a batch of image pairs (use_intrinsics_in_verification=True path).
 *
 * Keypoints of all images: d_kp_xy[n_img][kmax][2] float32 pixels; d_intrinsics[n_img][3] = (f, u0, v0)
 * (Cal3Bundler with k1 = k2 = 0). Putatives per pair: d_match_idx[n_pairs][mcap][2] uint32 keypoint indices
 * and d_match_count[n_pairs] (exactly the matcher's output). Threshold thr_px / max(f1, f2) in normalized
 * coordinates on the squared Sampson distance, success probability `prob`, at most `max_iters` hypotheses
 * (checked per batch of 64); `seed` and the pair id key the deterministic sampling of pair p: d_pair_ids[p]
 * when d_pair_ids is non-NULL (e.g. all 0 to reproduce one-pair calls), else pair_id_base + p.
 * Model selection `scoring` (ransac.py:58 robust_estimation_type): GTSFM_RANSAC_SCORING_MSAC for USAC_* (the default
 * USAC_ACCURATE scores models by MSAC: sum of min(squared Sampson error, thr^2)), each term quantised to
 * floor(e * 2^16 / thr^2) (65536 for an outlier) so the sum is exact in any order; GTSFM_RANSAC_SCORING_RANSAC for
 * cv2 RANSAC (inlier count). Local optimisation keeps a refit by the same criterion.
 * Outputs per pair: E, R (i2Ri1) row-major 3x3, unit t (i2ti1), inlier count, status (0 ok, 1 fewer than
 * 6 putatives, 2 no model), number of hypotheses evaluated (d_n_hyp may be NULL), number of candidate models scored
 * (the real 5-point solutions of those hypotheses; d_n_models may be NULL; a measurement output with no reference
 * counterpart, it prices the RANSAC FLOP count of SURVEY.md §8(d)) and the inlier mask d_inlier_mask[n_pairs][mcap]
 * over the putatives in matcher order. mcap < 2^19, and mcap <= 65535 with MSAC (the selection key's widths):
 * GTSFM_ERR_ARG otherwise.
 * ---------------------------------------------------------------------------------------------- */
size_t gtsfm_ransac_workspace_bytes(int n_pairs, int mcap);

#define GTSFM_RANSAC_SCORING_RANSAC 0 /* most inliers wins (cv2 RANSAC) */
#define GTSFM_RANSAC_SCORING_MSAC 1   /* lowest truncated-quadratic cost wins (USAC_ACCURATE's MSAC score) */

int gtsfm_ransac_E_batched(const float* d_kp_xy, const double* d_intrinsics, int n_img, int kmax,
                           const int* d_pairs, int n_pairs, const uint32_t* d_match_idx,
                           const int* d_match_count, int mcap, double thr_px, double prob, int max_iters,
                           int scoring, uint64_t seed, int pair_id_base, const int* d_pair_ids, void* d_workspace,
                           size_t workspace_bytes, double* d_E, double* d_R, double* d_t, int* d_n_inliers, int* d_status,
                           int* d_n_hyp, int* d_n_models, uint8_t* d_inlier_mask, void* stream);

/* ----------------------------------------------------------------------------------------------
 * Verifier, fundamental-matrix path (use_intrinsics_in_verification=False). Replaces Ransac.estimate_F
 * (gtsfm/frontend/verifier/ransac.py:84-111: cv2.findFundamentalMat(FM_RANSAC, thr_px, 0.999999, 1e6)) and the
 * F branch of OpencvVerifierBase.verify (opencv_verifier_base.py:90-109: E = K2^T F K1, recoverPose on the
 * K-normalised inliers). Same inputs as gtsfm_ransac_E_batched; pixel coordinates are used for estimation.
 * 7-point RANSAC for M >= 15, LMedS for 8 <= M < 15, normalised 8-point refit on the inliers.
 * Outputs per pair: F (F33 = 1), E, R (i2Ri1), unit t (i2ti1), inlier count, status (0 ok, 1 fewer than 8
 * putatives, 2 no model), hypotheses drawn (d_n_hyp may be NULL), inlier mask d_inlier_mask[n_pairs][mcap].
 * ---------------------------------------------------------------------------------------------- */
size_t gtsfm_ransac_F_workspace_bytes(int n_pairs, int mcap);

int gtsfm_ransac_F_batched(const float* d_kp_xy, const double* d_intrinsics, int n_img, int kmax,
                           const int* d_pairs, int n_pairs, const uint32_t* d_match_idx,
                           const int* d_match_count, int mcap, double thr_px, double prob, int max_iters,
                           uint64_t seed, int pair_id_base, const int* d_pair_ids, void* d_workspace,
                           size_t workspace_bytes, double* d_F, double* d_E, double* d_R, double* d_t,
                           int* d_n_inliers, int* d_status, int* d_n_hyp, uint8_t* d_inlier_mask, void* stream);

/* ----------------------------------------------------------------------------------------------
 * Two-view triangulation + bundle adjustment. Replaces TwoViewEstimator.bundle_adjust and the run_2view branch
 * that calls it (gtsfm/two_view_estimator.py:101-208, 311-337; gtsam.triangulatePoint3 + the 2-view
 * BundleAdjustmentOptimizer, bundle/bundle_adjustment.py:269-275, 359-419), batched over pairs; the restatement is
 * oracle/ba2.c (calibrations held fixed; the reference's sigma 1e-5 prior pins them).
 * Inputs: the verifier's keypoints / intrinsics / pairs / putatives exactly as gtsfm_ransac_E_batched takes them,
 * its inlier mask d_in_mask[n_pairs][mcap] (the pre-BA verified rows), i2Ri1 d_R_in[n_pairs][9], unit i2ti1
 * d_t_in[n_pairs][3] and status d_status_in (0 = verified). Optional relative-pose priors (two_view_estimator.py:165,
 * 192: bundle_adjust's i2Ti1_prior): d_prior_Rt[n_pairs][12] = the prior's i2Ti1 (R row-major, then t) and
 * d_prior_sigmas[n_pairs][6] its sigmas (PosePrior.covariance, rotation first); a pair with sigma[0] <= 0 has none,
 * both NULL = no priors. A prior initialises the second camera and adds BetweenFactorPose3(X0, X1, prior^-1)
 * (bundle_adjustment.py:136-152). Per pair with status 0 and >= min_inliers verified rows:
 * every verified row is triangulated (DLT + LM point refinement, cheirality, reprojection < tri_thresh px), the
 * 2-view BA runs (Huber 1.345 on 1 px, X0 prior 0.1, first-point prior 0.1, Levenberg-Marquardt <= max_iters
 * iterations), and rows whose two reprojections stay < reproj_thresh px survive (filter_landmarks).
 * Outputs: d_R_out / d_t_out (post-BA i2Ri1, unit i2ti1; the inputs when BA did not produce a pose),
 * d_out_mask[n_pairs][mcap] (post-BA verified rows; the input mask when BA did not run), d_n_out (its count),
 * d_status_out (0 BA ok, 1 no track triangulated, 2 no track valid after BA, 3 not run), d_iters (LM iterations,
 * may be NULL).
 * ---------------------------------------------------------------------------------------------- */
size_t gtsfm_ba2_workspace_bytes(int n_pairs, int mcap);

int gtsfm_ba2_batched(const float* d_kp_xy, const double* d_intrinsics, int n_img, int kmax, const int* d_pairs,
                      int n_pairs, const uint32_t* d_match_idx, const int* d_match_count, int mcap,
                      const uint8_t* d_in_mask, const double* d_R_in, const double* d_t_in, const int* d_status_in,
                      const double* d_prior_Rt, const double* d_prior_sigmas, int min_inliers, int max_iters,
                      double reproj_thresh, double tri_thresh, void* d_workspace,
                      size_t workspace_bytes, double* d_R_out, double* d_t_out, uint8_t* d_out_mask, int* d_n_out,
                      int* d_status_out, int* d_iters, void* stream);

/* ----------------------------------------------------------------------------------------------
 * Verified-correspondence compaction + inlier-support filter (the device half of the hand-off to the host).
 * d_n_inliers are the rows of d_inlier_mask each pair keeps (the verifier's counts, or gtsfm_ba2_batched's post-BA
 * counts with its mask); inlier_ratio = d_n_inliers / d_match_count unless d_ratio_inliers (may be NULL) gives the
 * count the ratio is taken on (the reference keeps the pre-BA ratio after BA: two_view_estimator.py:326-327).
 * Replaces, for every pair at once: v_corr_idxs = match_indices[mask == 1] and inlier_ratio = mean(mask)
 * (gtsfm/frontend/verifier/opencv_verifier_base.py:98-101) and InlierSupportProcessor.run_inlier_support
 * (gtsfm/frontend/inlier_support_processor.py:73-87: fail iff ratio < min_inlier_ratio or 0 < n < min_inliers).
 * Inputs are the matcher's d_match_idx[n_pairs][mcap][2] / d_match_count and the verifier's mask, status and inlier
 * counts. Outputs: d_offsets[n_pairs + 1] (exclusive scan of the rows each pair contributes: n_inliers when status is
 * 0, else 0), d_v_corr[offsets[p] .. offsets[p+1])[2] uint32 = pair p's inlier putatives in matcher order (rows past
 * `capacity` are not written; capacity = sum of match counts always suffices), d_isp_ok[n_pairs] = 1 iff the pair
 * verified and passes the inlier-support filter.
 * ---------------------------------------------------------------------------------------------- */
int gtsfm_compact_verified(const uint32_t* d_match_idx, const int* d_match_count, int mcap,
                           const uint8_t* d_inlier_mask, const int* d_status, const int* d_n_inliers,
                           const int* d_ratio_inliers, int n_pairs, int min_inliers, double min_inlier_ratio,
                           int* d_offsets, uint32_t* d_v_corr, int capacity, uint8_t* d_isp_ok, void* stream);

/* ----------------------------------------------------------------------------------------------
 * Squared Sampson distances. Replaces gtsfm/utils/verification.py:170-214 compute_epipolar_distances_sq_sampson (the
 * two-view report's ground-truth correspondence metric, gtsfm/utils/metrics.py:99-128), batched over pairs:
 * row r (of n_rows) pairs d_x1[r] (x, y) with d_x2[r] under matrix d_F[d_row_pair[r]] (row-major 3x3, n_mats of them):
 *   d_out[r] = (x2^T F x1)^2 / ((F x1)_x^2 + (F x1)_y^2 + (F^T x2)_x^2 + (F^T x2)_y^2).
 * precision GTSFM_SAMPSON_F64: float64 (the reference's numpy arithmetic). GTSFM_SAMPSON_F32_VERIFIER: the fp32 FMA
 * expression the essential-matrix RANSAC thresholds (its inlier test is d_out <= thr^2), for pinning the verifier.
 * ---------------------------------------------------------------------------------------------- */
#define GTSFM_SAMPSON_F64 0
#define GTSFM_SAMPSON_F32_VERIFIER 1

int gtsfm_sampson_sq_batched(const double* d_F, int n_mats, const int* d_row_pair, const double* d_x1,
                             const double* d_x2, int n_rows, int precision, double* d_out, void* stream);

/* ----------------------------------------------------------------------------------------------
 * Detector-descriptor: SIFT (OpenCV defaults) + top-k by response over a batch of same-sized images.
 *
 * d_images[n_img][H][W][channels] uint8, channels 1 (gray) or 3 (RGB, converted like cv.COLOR_RGB2GRAY).
 * d_masks[n_img][H][W] uint8 or NULL: as detectAndCompute(gray, image.mask) (reference sift.py:47), a keypoint is
 * dropped when its pixel mask[(int)(y + 0.5)][(int)(x + 0.5)] is 0, before the top-k.
 * Outputs per image, rows 0..count-1 valid, ordered by descending response:
 *   d_xy[n_img][max_kpts][2]   keypoint (x, y) in pixels (x right, y down, origin top-left corner)
 *   d_attr[n_img][max_kpts][3] (size, angle in degrees, response) as cv.KeyPoint
 *   d_desc[n_img][max_kpts][128] float32 descriptors with integer values in [0, 255]
 *   d_counts[n_img] = min(#keypoints, max_kpts); d_n_detected[n_img] (may be NULL) = #keypoints before top-k
 *   (after the mask).
 * Limits: 16 <= H, W < 4096, max_kpts <= 8192.
 * ---------------------------------------------------------------------------------------------- */
size_t gtsfm_sift_workspace_bytes(int n_img, int H, int W, int max_kpts);

int gtsfm_sift_batched(const uint8_t* d_images, const uint8_t* d_masks, int n_img, int H, int W, int channels,
                       int max_kpts, void* d_workspace, size_t workspace_bytes, float* d_xy, float* d_attr, float* d_desc,
                       int* d_counts, int* d_n_detected, void* stream);

/* ----------------------------------------------------------------------------------------------
 * SuperPoint detector-descriptor. Replaces SuperPointDetectorDescriptor.detect_and_describe
 * (gtsfm/frontend/detector_descriptor/superpoint.py:48-74) and the network it wraps
 * (thirdparty/SuperGluePretrainedNetwork/models/superpoint.py:145-202), batched over n same-sized images
 * d_images[n][H][W][C] (C = 1 gray or 3 RGB -> cv COLOR_RGB2GRAY fixed point), scaled by 1/255.
 * d_weights: packed fp32 blob of gtsfm_superpoint_weights_floats() floats, layers in the order
 *   conv1a, conv1b, conv2a, conv2b, conv3a, conv3b, conv4a, conv4b, [convPa | convDa], convPb, convDb
 * each as W[k*k][cin][cout_pad] (W[ky*k+kx][ci][co] = torch weight[co][ci][ky][kx]) followed by bias[cout_pad];
 * (k, cin, cout_pad) = (3,1,64) (3,64,64) (3,64,64) (3,64,64) (3,64,128) (3,128,128) (3,128,128) (3,128,128)
 * (3,128,512: Pa in 0..255, Da in 256..511) (1,256,128: 65 used) (1,256,256); padded outputs are zero.
 * Detection: softmax over 65, 8x8 depth-to-space, simple_nms(nms_radius), score > keypoint_threshold, border
 * remove_borders; d_masks[n][H][W] u8 or NULL: as Keypoints.filter_by_mask (reference superpoint.py:68-70), a
 * detection at pixel (x, y) is kept iff mask[y][x] == 1, before the top-k; the max_kpts highest scores are kept
 * (ties by raster order) and emitted in raster order (the reference's own order when max_kpts >= detections).
 * Outputs: d_xy[n][max_kpts][2] (x, y) float, d_scores[n][max_kpts], d_desc[n][max_kpts][256] unit-norm,
 * d_count[n], d_n_detected[n] (detections after border and mask, before the top-k; may be NULL).
 * ---------------------------------------------------------------------------------------------- */
size_t gtsfm_superpoint_weights_floats(void);

size_t gtsfm_superpoint_workspace_bytes(int n, int H, int W, int max_kpts);

int gtsfm_superpoint_batched(const uint8_t* d_images, const uint8_t* d_masks, int n, int H, int W, int C,
                             const float* d_weights, int max_kpts, float keypoint_threshold, int nms_radius,
                             int remove_borders, void* d_workspace, size_t workspace_bytes, float* d_xy,
                             float* d_scores, float* d_desc, int* d_count, int* d_n_detected, void* stream);

/* ----------------------------------------------------------------------------------------------
 * SuperGlue matcher. Replaces SuperGlueMatcher.match (gtsfm/frontend/matcher/superglue_matcher.py:43-111) and
 * the network it wraps (thirdparty/SuperGluePretrainedNetwork/models/superglue.py:228-283), batched over pairs.
 * Features of all images: d_kp[n_img][kmax][2] (x, y) float, d_scores[n_img][kmax], d_desc[n_img][kmax][256],
 * d_counts[n_img], d_image_hw[n_img][2] = (H, W); kmax a multiple of 64. Pairs d_pairs[n_pairs][2] (both sides
 * must hold >= 1 keypoint: the reference returns no matches for an empty side before running the network).
 * d_weights: gtsfm_superglue_weights_floats(n_layers) floats (layout in superglue.hip: W^T[cin][cout] per 1x1 conv,
 * eval BatchNorm folded to scale/shift, q/k/v/merge weights permuted head-major). GNN layer l is 'self' for even l,
 * 'cross' for odd l. Outputs: matches (i, j) with i ascending in d_out_idx[n_pairs][kmax][2] uint32, counts
 * d_out_count[n_pairs], and the matching scores of image-0 keypoints d_out_mscores[n_pairs][kmax] (may be NULL).
 * ---------------------------------------------------------------------------------------------- */
size_t gtsfm_superglue_weights_floats(int n_layers);

size_t gtsfm_superglue_workspace_bytes(int n_pairs, int kmax);

int gtsfm_superglue_batched(const float* d_kp, const float* d_scores, const float* d_desc, const int* d_counts,
                            const int* d_image_hw, int n_img, int kmax, const int* d_pairs, int n_pairs,
                            const float* d_weights, int n_layers, int sinkhorn_iters, float match_threshold,
                            void* d_workspace, size_t workspace_bytes, uint32_t* d_out_idx, int* d_out_count,
                            float* d_out_mscores, void* stream);

/* Inspection hook (the reference keeps this matrix internal: superglue.py:261-263 `scores`): after a
 * gtsfm_superglue_batched call, writes pair `pair`'s final log-assignment matrix (log_optimal_transport's output, the
 * Sinkhorn result + the normalisation) from that call's workspace into d_out[(kmax + 1)][(kmax + 1)]: rows 0..m,
 * columns 0..n (the last of each being the dustbin), NaN elsewhere. Same n_pairs / kmax as the call. */
int gtsfm_superglue_log_assignment(const void* d_workspace, size_t workspace_bytes, int n_pairs, int kmax, int pair,
                                   float* d_out, void* stream);

/* ---- Retrieval (f3): NetVLAD global-descriptor similarity + top-k image pairs ---------------------------------- */

/* Replaces NetVLADRetriever.compute_similarity_matrix (gtsfm/retriever/netvlad_retriever.py:77-107) together with
 * _compute_similarity_subblock (:109-134, the einsum "id,jd->ij" per block pair block_j >= block_i) and
 * _aggregate_subblocks (:136-149). d_desc: [n_img][dim] f32 global descriptors; d_sim: [n_img][n_img] f32, fully
 * written: the dot product where block(j) >= block(i) (block = index / blocksize), 0 elsewhere, as the reference's
 * zero-initialised aggregate. fp32 accumulation (summation order differs from torch: parity is a tolerance). */
int gtsfm_retrieval_similarity(const float* d_desc, int n_img, int dim, int blocksize, float* d_sim, void* stream);

/* Replaces pairs_from_score_matrix (netvlad_retriever.py:196-228). d_scores: [n_rows][n_cols] f32. d_invalid:
 * [n_rows][n_cols] u8 (nonzero = invalid), or NULL for compute_pairs_from_similarity_matrix's mask (:164-167: every
 * entry not strictly above the diagonal is invalid). k = min(num_select, n_rows) (:213-215; k > n_cols is
 * GTSFM_ERR_ARG, as torch.topk raises); scores < min_score are invalid when use_min_score != 0. For row i,
 * d_out_pairs[(i * k + r) * 2 + {0,1}] = (i, j_r) for r < d_row_count[i]: the finite entries of torch.topk(row, k) in
 * rank order (NaN ranks first and takes a slot but is not emitted; equal scores by ascending column, an order torch
 * leaves unspecified). The reference's pair list is the rows concatenated in order. d_scores is read only (the
 * reference masks its argument in place). */
int gtsfm_retrieval_pairs(const float* d_scores, int n_rows, int n_cols, const unsigned char* d_invalid, int num_select,
                          float min_score, int use_min_score, int* d_out_pairs, int* d_row_count, void* stream);

/* ---- Global descriptor (f3): NetVLAD ---------------------------------------------------------------------------- */

/* Replaces NetVLADGlobalDescriptor.describe (gtsfm/frontend/global_descriptor/netvlad_global_descriptor.py:27-46)
 * and the network it runs (thirdparty/hloc/netvlad.py:160-191), batched over n same-sized RGB images
 * d_images[n][H][W][3] u8 (describe()'s image.value_array). Per image: x = clamp(u / 255 * 255, 0, 255) - mean,
 * VGG16 features[:-2] (13 conv3x3 + ReLU except the last, 2x2 max-pools after convs 2, 4, 7, 10, floor), per-location
 * L2 pre-normalisation, NetVLADLayer (K = 64 clusters, D = 512: softmax(score_proj x), residual sums, intra-norm,
 * d-major flatten, L2), then (whiten != 0) the 32768 -> 4096 whitening Linear and L2.
 * d_weights: gtsfm_netvlad_weights_floats() floats:
 *   mean[4] (averageImage RGB, 1 pad); per conv l = 0..12: W[9][cin][cout] (W[ky*3+kx][ci][co] = torch
 *   backbone weight[co][ci][ky][kx]) then bias[cout], (cin, cout) = (3,64) (64,64) (64,128) (128,128) (128,256)
 *   (256,256) (256,256) (256,512) (512,512) x 5; score_proj[64][512]; centers[512][64]; whiten W[4096][32768]
 *   (nn.Linear's weight, row = output); whiten b[4096].
 * Outputs: d_vlad[n][32768] (may be NULL when whiten != 0) and d_desc[n][4096] (whiten != 0). fp32-accurate
 * arithmetic (convolutions as split-bf16 MFMA products, the rest fp32): parity with the reference is a tolerance. */
size_t gtsfm_netvlad_weights_floats(void);

size_t gtsfm_netvlad_workspace_bytes(int n, int H, int W);

int gtsfm_netvlad_batched(const uint8_t* d_images, int n, int H, int W, int C, const float* d_weights, int whiten,
                          float* d_vlad, float* d_desc, void* d_workspace, size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GTSFM_HIP_H_ */
