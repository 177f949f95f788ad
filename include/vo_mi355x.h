/*
 * vo_mi355x.h -- C ABI of the MI355X-native extract -> match -> pose hot path.
 *
 * Drop-in boundary for the reference's per-frame path (Bohdanok/ACS_Visual_Odometry,
 * the `VisualOdometry` binary).  The reference exposes only C++ classes (no C ABI);
 * each entry point below replaces the reference call named in its comment.  The C++
 * facade `include/VisualOdometry.hpp` and the Python facade
 * `acs_visual_odometry_amd.VisualOdometry` re-expose these under the reference's
 * method names.
 *
 * Conventions
 *  - return 0 on success, < 0 on error (vo_strerror); no exception crosses the ABI.
 *  - all pointers are caller-owned HOST memory unless the name ends in _device.
 *  - a vo_ctx is bound to one GPU and one HIP stream; it is not thread-safe
 *    (one ctx per host thread / GPU, like one VisualOdometry object per run).
 *  - keypoints are (x = column, y = row), raster (row, col) ascending order.
 *  - descriptors are 512 test bits as 8 x uint64, bit t in word t/64, LSB first;
 *    vo_unpack_descriptor gives the reference's byte-per-test layout.
 */
#ifndef VO_MI355X_H
#define VO_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VO_ABI_VERSION 2   /* 2: vo_config gained rng_mode (round 5); a binary built against
                              version 1 has a shorter vo_config and must be rebuilt */

/* error codes */
#define VO_OK                 0
#define VO_ERR_ARG           (-1)
#define VO_ERR_HIP           (-2)
#define VO_ERR_NO_DEVICE     (-3)   /* VisualOdometry.cpp:17-19 throws "No OpenCL devices" */
#define VO_ERR_CAPACITY      (-4)
#define VO_ERR_STATE         (-5)
#define VO_ERR_IO            (-6)   /* image file missing or not decodable (cv::imread -> empty) */
#define VO_ERR_INTERNAL      (-7)   /* a device consistency check failed (VO_STATUS_INCONSISTENT
                                       frames) or a bounded in-kernel wait timed out (the per-frame
                                       call's fused select / fused RANSAC); vo_device_error_count
                                       counts both.  Results of the call are not those of the
                                       reference.  Sticky until vo_reset. */
#define VO_ERR_DEGENERATE_E  (-10)  /* PoseUpdate.hpp:71-73 throws "Degenerate essential matrix" */

/* per-frame status (VisualOdometry.cpp:68-189) */
#define VO_STATUS_OK            0   /* pose updated                                  */
#define VO_STATUS_FIRST         1   /* frame 0: identity pushed (:58)                */
#define VO_STATUS_MISSING       2   /* image failed to load (:77-82), T_curr pushed  */
#define VO_STATUS_FEW_MATCHES   3   /* < 8 matches (:108-115), flipZ*T_curr pushed   */
#define VO_STATUS_FEW_INLIERS   4   /* < 8 model inliers (:147-153)                  */
#define VO_STATUS_DEGENERATE    5   /* getPose threw (countNonZero(E) < 5)           */
#define VO_STATUS_OVERFLOW      6   /* (not produced since round 3: boundary bins of any size are ranked) */
#define VO_STATUS_STALLED       7   /* frame pipeline: this frame's extract never signalled */
#define VO_STATUS_INCONSISTENT  8   /* the stencil's histogram disagrees with its keys, or the top-N
                                       select emitted other than min(C, N) keypoints: the frame is
                                       treated as having 0 keypoints and the call returns
                                       VO_ERR_INTERNAL (never expected; a library defect) */

typedef struct vo_ctx vo_ctx;

typedef struct { int32_t x, y; } vo_kp;
typedef struct { int32_t prev, cur; } vo_match_t;

typedef struct {
    int width, height;
    int max_kpts;             /* N = 2000      feature_extraction_parallel_GPU.cpp:235 */
    int nms_k;                /* 3             feature_extraction_parallel_GPU.cpp:235 */
    float resp_thr;           /* 20000         corner_detection_parallel_GPU.h:25      */
    int border_row;           /* 35            corner_detection_parallel_GPU.cpp:157   */
    int border_col;           /* 37            corner_detection_parallel_GPU.cpp:157   */
    float ratio;              /* 0.75          VisualOdometry.cpp:35                   */
    int match_bits;           /* 32 (reference quirk 1) or 512 (matching_serial.cpp)   */
    double ransac_p;          /* 0.99          VisualOdometry.cpp:130                  */
    double sampson_thr;       /* 1.0           VisualOdometry.cpp:130                  */
    int ransac_chunk_threads; /* T             ransac.cpp:152-157 (CLI num_threads)    */
    uint64_t seed;            /* RANSAC sampler seed (replaces std::random_device)     */
    double K[9];              /* PoseUpdate.hpp:36-39                                  */
    int device;               /* HIP device ordinal                                    */
    int frame_batch;          /* frames per extract batch / pose-pass window (1..128);
                                 0 = default 64.  Results do not depend on it.         */
    int rng_mode;             /* RANSAC sampler (ransac.cpp:137,142):
                                 VO_RNG_SPLITMIX (default): Floyd samples from splitmix64, drawn
                                   on the device per hypothesis (the throughput mode);
                                 VO_RNG_MT19937: the reference's own sampler, std::sample(data, 8,
                                   rng) with std::mt19937 rng(seed32) per frame -- seed32 = the low
                                   32 bits of the frame seed (of `seed` in the stage calls), where
                                   the reference seeds std::random_device{}() -- drawn on the host
                                   once the frame's match count is known (a host round trip per
                                   pose pass).  A reference build seeded with seed32 draws the same
                                   hypotheses. */
} vo_config;
#define VO_RNG_SPLITMIX 0
#define VO_RNG_MT19937  1

/* Fill the reference defaults for a width x height stream. */
void vo_config_default(vo_config* cfg, int width, int height);

/* VisualOdometry::VisualOdometry(kernel_filename, num_threads)  VisualOdometry.h:23.
 * Allocates every device buffer once (the reference re-allocates per frame). */
int  vo_create(const vo_config* cfg, vo_ctx** out);
void vo_destroy(vo_ctx* ctx);
const char* vo_strerror(int code);
int  vo_abi_version(void);

/* VisualOdometry::compute_descriptor_with_key_points  VisualOdometry.h:25-26
 * (-> feature_extraction_manager_with_points, feature_extraction_parallel_GPU.cpp:194).
 * kps: max_kpts entries; desc: max_kpts * 8 words; blurred (optional): W*H bytes. */
int  vo_extract(vo_ctx* ctx, const uint8_t* gray, size_t stride, vo_kp* kps, uint64_t* desc,
                int* n, uint8_t* blurred);

/* Dense response map R (W*H f32, 0 outside [2,H-3]x[2,W-3] and below threshold):
 * gradient_convolution + shitomasi_response, kernels/feature_extraction_kernel_functions.c:43-120. */
int  vo_response(vo_ctx* ctx, const uint8_t* gray, size_t stride, float* R);

/* VisualOdometry::match_descriptors  VisualOdometry.h:27-29
 * (-> matchCustomBinaryDescriptorsThreadPool, feature_matching_parallel.cpp:49-113). */
int  vo_match(vo_ctx* ctx, const uint64_t* d_prev, int n_prev, const uint64_t* d_cur, int n_cur,
              vo_match_t* out, int* m);

/* Ransac::run(model, data, p, thr, T, pool)  ransac.hpp:42-47, + FundamentalMatrix::getMatrix/
 * getInliers (ransac.hpp:31,33).  pts: m x (x1,y1,x2,y2).  seed: sampler seed for this call.
 * F: refit model (valid iff *fitted).  inlier_idx (m entries, optional): bestInlierSet as
 * indices into pts.  counts (optional, 2000 entries): inliers of hypothesis k for
 * k < *n_evaluated. */
int  vo_ransac_F(vo_ctx* ctx, const double* pts, int m, uint64_t seed, double F[9],
                 int* fitted, int32_t* inlier_idx, int* n_inl, int* best_k, int* n_evaluated,
                 int32_t* counts);

/* Ransac::run(model, data, probability, sampsonThreshold, numThreads, pool)  ransac.hpp:42-47,
 * ransac.cpp:120-194, with the call's own parameters: pts m x (x1,y1,x2,y2) (m >= 8; the reference
 * is undefined below 8), the chunk drop of num_threads chunks (quirk 7), the sampler seed of this
 * call.  *fitted = 1: model.fit(bestInlierSet) ran (>= 8 inliers) and F is its F; 0: the model
 * keeps its previous F and inliers (quirk 9; F untouched).  inlier_idx (optional, m entries): the
 * best hypothesis' inliers in data order.  VO_ERR_CAPACITY if the probability's initial
 * iteration bound exceeds the context's 2000 hypothesis slots. */
int  vo_ransac_run(vo_ctx* ctx, const double* pts, int m, double probability, double sampson_thr,
                   int num_threads, uint64_t seed, double F[9], int* fitted, int32_t* inlier_idx,
                   int* n_inl, int* n_evaluated);

/* FundamentalMatrix::fit(sample) -> computeFundamentalMatrix  ransac.cpp:63-99: normalized
 * least-squares F of all n >= 8 correspondences (pts n x (x1,y1,x2,y2)), rank 2 enforced. */
int  vo_fit_F(vo_ctx* ctx, const double* pts, int n, double F[9]);

/* PoseUpdate::getPose(F, points1, points2, scale)  PoseUpdate.hpp:61-62.
 * p1/p2: n x 2 f32.  counts4 (optional): positive-depth count per candidate
 * {R1,t},{R1,-t},{R2,t},{R2,-t}.  Returns VO_ERR_DEGENERATE_E where the reference throws. */
int  vo_pose(vo_ctx* ctx, const double F[9], const float* p1, const float* p2, int n,
             double scale, double R[9], double t[3], int32_t* counts4);

/* Ground truth for the trajectory loop's scale (VisualOdometry.cpp:161-162): n rows of
 * 12 doubles (KITTI 3x4 row-major).  Without it the scale is 1.  The rows are copied into a
 * pinned staging buffer before the call returns (the caller's array may be freed) and reach the
 * device asynchronously, ahead of every later call's kernels; like vo_set_sequence_starts, the
 * call does not wait for the GPU unless the row count outgrows the device buffer. */
int  vo_set_ground_truth(vo_ctx* ctx, const double* poses12, int n);

/* Independent sequences in one frame stream (config 5 on one GPU): frames starts[0..n) (counted
 * since vo_reset, strictly ascending, >= 1) each begin a new sequence -- the trajectory state is
 * reset there as at the start of a new VisualOdometry::run (identity pose, no model, desc1 = that
 * frame; VisualOdometry.cpp:46-66) -- so a batched call over several sequences' frames, with their
 * ground-truth rows concatenated in the same order, returns each sequence's own rows while the
 * extract of the next sequence overlaps the last pose passes of the previous one.  n = 0: one
 * sequence.  Kept across vo_reset. */
int  vo_set_sequence_starts(vo_ctx* ctx, const int32_t* starts, int n);

/* Sequence shards (one sequence split over GPUs; acs_visual_odometry_amd/shard.py).  A shard's
 * stream starts at frame `origin` of its sequence: its first frame starts the trajectory as
 * VisualOdometry.cpp:57-66 do (the halo of the shard: identity pose, no model), and the RANSAC
 * sampler of the stream's first sequence counts frames from origin, so every frame draws the
 * hypotheses it draws in the unsplit run.  Kept across vo_reset; 0 = an ordinary stream. */
int  vo_set_frame_origin(vo_ctx* ctx, int origin);
/* Frames whose keypoints, descriptors and trajectory records stay resident on the device (the
 * ring: 4096 by default, VO_RING_SLOTS): vo_rechain reaches back this far, so a shard may hold at
 * most this many frames.  Returns the count (> 0) or an error code. */
int  vo_ring_slots(vo_ctx* ctx);
/* T_curr after the last committed frame (VisualOdometry.cpp:184, 4x4 row-major). */
int  vo_trajectory_state(vo_ctx* ctx, double Tcurr[16]);
/* The trajectory chain (VisualOdometry.cpp:161-186) of committed frames [f0, f0 + n) (counted since
 * vo_reset) again, from T_curr = T_in instead of the chain the stream ran: the rows a shard's frames
 * get in the unsplit run once its predecessor's T_curr is known.  The frames' trajectory records
 * must still be in the ring (f0 >= frames - ring slots); T_curr is left at the chain's end.
 * poses_out: n x 12 (host, optional). */
int  vo_rechain(vo_ctx* ctx, const double T_in[16], int f0, int n, double* poses_out);

/* One iteration of VisualOdometry::run's loop (VisualOdometry.cpp:68-189): frame in,
 * pose out.  gray == NULL marks a missing image.  pose_out: 12 doubles, the row the
 * reference appends to estimated_poses.  info (optional, 8 ints): n_kpts, n_matches,
 * n_inliers, best_k, n_evaluated, fitted, 0, 0. */
int  vo_process_frame(vo_ctx* ctx, const uint8_t* gray, size_t stride, double pose_out[12],
                      int* status, int32_t* info);

/* Batched, device-resident variant: nframes frames already in HBM at
 * d_frames + f * frame_bytes (dense W x H u8).  Frames are extracted frame_batch at a time
 * on one queue and posed in windows of frame_batch frames on another (each frame matched
 * speculatively against its predecessor; a frame after a skipped one is re-run), with one
 * host synchronisation per chunk of ring - 1 = 4095 frames (more only after skipped frames).  Results
 * are those of nframes vo_process_frame calls.  poses_out: nframes*12, status_out: nframes,
 * info_out: nframes*8 (all host, optional). */
int  vo_process_frames_device(vo_ctx* ctx, const uint8_t* d_frames, size_t frame_bytes, int nframes,
                              double* poses_out, int* status_out, int32_t* info_out);

/* Batched extract only (SURVEY config 2; feature_extraction_manager_with_points over many
 * frames): nframes device-resident frames, frame_batch per launch.  Optional host outputs:
 * kps (nframes * max_kpts), desc (nframes * max_kpts * 8 words), n_kps (nframes).  The ring
 * slots are reused, so the trajectory state is reset (as by vo_reset) before and after. */
int  vo_extract_frames_device(vo_ctx* ctx, const uint8_t* d_frames, size_t frame_bytes, int nframes,
                              vo_kp* kps, uint64_t* desc, int32_t* n_kps);

/* Host-frame streaming variant (the drop-in path of VisualOdometry::run, whose loop reads one
 * image per iteration, VisualOdometry.cpp:68-189): nframes dense W x H u8 frames in HOST memory
 * at frames + f * frame_bytes.  Batch k + 1's H2D copy runs on a copy queue while batch k is
 * extracted and earlier windows are posed; nothing synchronises the host until the chunk ends.
 * Pinned memory (vo_host_alloc, or the caller's own hipHostMalloc / hipHostRegister) is DMA'd
 * directly; pageable memory is registered for the duration of the call, or staged through a
 * pinned ring if registration fails.  Results are those of nframes vo_process_frame calls. */
int  vo_process_frames_host(vo_ctx* ctx, const uint8_t* frames, size_t frame_bytes, int nframes,
                            double* poses_out, int* status_out, int32_t* info_out);

/* cv::imread(path, cv::IMREAD_GRAYSCALE)  VisualOdometry.cpp:65,76, for PNG (any bit depth /
 * colour type, Adam7) and binary PGM.  Writes width x height u8 pixels to out when out != NULL
 * and cap >= width * height (VO_ERR_CAPACITY otherwise; the dimensions are always set on a
 * successful decode).  VO_ERR_IO where imread returns an empty Mat. */
int  vo_imread_gray(const char* path, uint8_t* out, size_t cap, int* width, int* height);

/* Pinned host memory for vo_process_frames_host sources. */
int  vo_host_alloc(vo_ctx* ctx, size_t bytes, void** hptr);
int  vo_host_free(vo_ctx* ctx, void* hptr);

/* Device memory helpers for callers without their own allocator (bench, tests). */
int  vo_device_alloc(vo_ctx* ctx, size_t bytes, void** dptr);
int  vo_device_free(vo_ctx* ctx, void* dptr);
int  vo_device_upload(vo_ctx* ctx, void* dptr, const void* src, size_t bytes);

/* The reference's RANSAC sampler, host only (no device needed): for k = 0 .. nhyp-1 the indices
 * (ascending) that the k-th std::sample(data.begin(), data.end(), std::back_inserter(sample), 8, rng)
 * of ransac.cpp:142 picks from m elements, rng = std::mt19937(seed32) constructed once
 * (ransac.cpp:137).  out: nhyp * 8 indices.  What VO_RNG_MT19937 uploads per frame. */
int  vo_reference_samples(uint32_t seed32, int m, int nhyp, int32_t* out);

/* Device consistency failures since vo_create / the last vo_reset (frames marked
 * VO_STATUS_INCONSISTENT by the top-N select, and timed-out bounded waits of the fused per-frame
 * kernels).  Waits for the context's queues.  The bench and the GPU tests assert it is 0. */
int  vo_device_error_count(vo_ctx* ctx, uint32_t* count);

/* Reset the trajectory state (frame counter, T_curr, model, prev descriptors). */
int  vo_reset(vo_ctx* ctx);

/* Per-kernel timing of vo_process_frames_device (HIP events on the stream each kernel runs on).
 * on: 0 off, 1 every launch of every kernel, 100+k only kernel k, on every 4th launch (an
 * event pair costs ~6 us of queue time, so the live timing samples).  times: average ms per
 * timed launch over the last call (-1 if not timed).  Returns the number written.
 * vo_last_kernel_stats also gives the frames per launch (frames of the call / launches). */
int  vo_last_kernel_times(vo_ctx* ctx, const char** names, float* ms, int cap);
int  vo_last_kernel_stats(vo_ctx* ctx, const char** names, float* ms_per_launch, float* frames_per_launch,
                          int cap);
int  vo_enable_kernel_timing(vo_ctx* ctx, int on);
/* The kernel symbol(s) stage k (numbered as vo_last_kernel_stats names them) launches on the
 * batched path of this context, as base names ("k_match"; the banded select:
 * "k_select_count,k_select_emit"): the rows of a rocprofv3 summary that belong to the stage. */
const char* vo_kernel_form(vo_ctx* ctx, int k);

/* desc512 (8 words) -> 512 bytes in {0,1}: the reference's byte-per-test layout
 * (desc[kp * 512 + t] = I(p1) > I(p2), kernels/feature_extraction_kernel_functions.c:223, read
 * back as vector<vector<uint8_t>> at FREAK_feature_descriptor_parallel_GPU.cpp:179,196-198). */
void vo_unpack_descriptor(const uint64_t words[8], uint8_t bytes[512]);

#ifdef __cplusplus
}
#endif
#endif
