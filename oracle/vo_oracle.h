/*
 * vo_oracle.h -- CPU ORACLE (test infrastructure only).
 *
 * Plain-C restatement of the reference's per-frame extract -> match -> pose path
 * (Bohdanok/ACS_Visual_Odometry, VisualOdometry binary).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker / the timed CPU baseline.  The product path
 * (acs_visual_odometry_amd/, libvo_mi355x.so) never links or calls it.
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - extract kernels (gradient/response/orientation/descriptor) are pinned against
 *     the reference's own OpenCL kernels, compiled from
 *     /root/reference/kernels/feature_extraction_kernel_functions.c by
 *     oracle/ref_kernels.mk into oracle/_ref/ and run on the GPU box by
 *     tests/test_ref_kernels.py (IEEE-strict build: bit-exact; stock build: ulp report).
 *   - blur (OpenCV GaussianBlur 8U bit-exact path), NMS/top-N, matcher, RANSAC,
 *     getPose depend on OpenCV/Eigen which are absent here: those stages are
 *     restated from the reference sources and pinned by analytic known-answer
 *     tests (tests/test_oracle_kat.py) -- parity unpinned against a reference run.
 *
 * Arithmetic follows SURVEY.md Appendix A.  Build with -ffp-contract=off.
 */
#ifndef VO_ORACLE_H
#define VO_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- configuration: same meaning as vo_config in include/vo_mi355x.h ---- */
typedef struct {
    int width, height;
    int max_kpts;            /* 2000   feature_extraction_parallel_GPU.cpp:235      */
    int nms_k;               /* 3      feature_extraction_parallel_GPU.cpp:235      */
    float resp_thr;          /* 20000  corner_detection_parallel_GPU.h:25           */
    int border_row;          /* 35     corner_detection_parallel_GPU.cpp:157        */
    int border_col;          /* 37     corner_detection_parallel_GPU.cpp:157        */
    float ratio;             /* 0.75   VisualOdometry.cpp:35                        */
    int match_bits;          /* 32     feature_matching_parallel.cpp:39-47 (512: matching_serial.cpp:24-40) */
    double ransac_p;         /* 0.99   VisualOdometry.cpp:130                       */
    double sampson_thr;      /* 1.0    VisualOdometry.cpp:130                       */
    int ransac_chunk_threads;/* T      ransac.cpp:152-157 (CLI thread count)        */
    uint64_t seed;           /* RANSAC sampler seed (replaces std::random_device)   */
    double K[9];             /* PoseUpdate.hpp:36-39                                */
    int rng_mode;            /* 0: Floyd / splitmix64 samples; 1: std::mt19937 + std::sample (ransac.cpp:137,142) */
} voo_config;
/* the reference's sampler (vo_oracle_mt.cpp): hypotheses k = 0 .. nhyp-1 of std::mt19937(seed32) */
void voo_mt_samples(uint32_t seed32, int m, int nhyp, int32_t* out);

void voo_config_default(voo_config* c, int width, int height);

/* ---- deterministic math (Appendix A.6 / A.8) ---- */
double voo_det_atan2(double y, double x);
double voo_det_sin(double x);
double voo_det_cos(double x);
uint64_t voo_mix64(uint64_t z);
void voo_sample8(uint64_t seed, int k, int m, int32_t out[8]);
uint64_t voo_frame_seed(uint64_t seed, int64_t frame);
int voo_ransac_maxit_update(int best, int n, double prob);   /* ransac.cpp:179-190 (glibc log/pow) */
int voo_ransac_maxit_initial(double prob);                    /* ransac.cpp:131 */

/* ---- extract (feature_extraction_manager_with_points, feature_extraction_parallel_GPU.cpp:194-306) ---- */
void voo_blur7(const uint8_t* src, size_t stride, int W, int H, uint8_t* dst);
void voo_gradients(const uint8_t* blurred, int W, int H, float* Jx, float* Jy, float* Jxy);
void voo_response(const uint8_t* blurred, int W, int H, float thr, float* R);
int  voo_nms_topn(const float* R, int W, int H, int k, int N, int brow, int bcol, int32_t* kps_xy);
int  voo_nms_candidates(const float* R, int W, int H, int k, int brow, int bcol);
void voo_orientation(const uint8_t* blurred, int W, int kx, int ky, float* ox, float* oy);
void voo_describe(const uint8_t* blurred, int W, int H, const int32_t* kps_xy, int n,
                  uint64_t* desc /* n*8 */, float* rot /* n*4 or NULL */);
int  voo_extract(const voo_config* c, const uint8_t* gray, size_t stride,
                 int32_t* kps_xy, uint64_t* desc, uint8_t* blurred_out /* or NULL */);

/* ---- match (matchCustomBinaryDescriptorsThreadPool, feature_matching_parallel.cpp:49-113) ---- */
int  voo_match(const uint64_t* d1, int n1, const uint64_t* d2, int n2, int match_bits, float ratio,
               int32_t* pairs /* 2*n1 */);

/* ---- RANSAC (Ransac::run, ransac.cpp:120-194) ---- */
typedef struct {
    double F[9];        /* refit model (valid iff fitted)                       */
    int fitted;         /* 1: model.fit(bestInlierSet) replaced the model        */
    int best_k;         /* index of the hypothesis that set bestInliers, or -1   */
    int best_count;
    int n_evaluated;    /* hypotheses evaluated (= final loop trip count)       */
    int n_inl;          /* |bestInlierSet|                                       */
} voo_ransac_result;

int  voo_fit_F(const double* pts, const int32_t* idx, int n, double F[9]);
int  voo_fit_F_warm(const double* pts, const int32_t* idx, int n, const double* Fb, double F[9]);
/* the refit's least-squares null vector of a 9x9 PSD S from warm start x0; returns 0 converged,
 * 1 certified in the numerical null space after 32 power steps, 2 cyclic-Jacobi fallback */
int  voo_ls_nullvec9(const double* S, const double* x0, double* f);
/* the refit's normal matrix A^T A of inliers idx (its fixed summation order) */
int  voo_refit_normal(const double* pts, const int32_t* idx, int n, double AtA_out[81]);
int  voo_fit_F8(const double* pts, const int32_t idx[8], double F[9]);
double voo_sampson(const double F[9], const double* p);
int  voo_ransac(const double* pts /* m*4: x1,y1,x2,y2 */, int m, double prob, double thr,
                int T, uint64_t seed, int32_t* counts /* >=2000 or NULL */,
                int32_t* inl_idx /* m or NULL */, voo_ransac_result* res);
int  voo_ransac_ex(const double* pts, int m, double prob, double thr, int T, uint64_t seed, int rng_mode,
                   int32_t* counts, int32_t* inl_idx, voo_ransac_result* res);

/* ---- pose (PoseUpdate::getPose, PoseUpdate.hpp:61-179) ---- */
#define VOO_OK 0
#define VOO_ERR_DEGENERATE_E (-10)
int  voo_pose(const double F[9], const double K[9], const float* p1, const float* p2, int n,
              double scale, double R[9], double t[3], int* counts4 /* 4 or NULL */);

/* ---- trajectory loop (VisualOdometry::run, VisualOdometry.cpp:38-193) ---- */
#define VO_STATUS_OK            0
#define VO_STATUS_FIRST         1
#define VO_STATUS_MISSING       2
#define VO_STATUS_FEW_MATCHES   3
#define VO_STATUS_FEW_INLIERS   4
#define VO_STATUS_DEGENERATE    5

typedef struct voo_vo voo_vo;
voo_vo* voo_vo_create(const voo_config* c);
void voo_vo_destroy(voo_vo* s);
/* per-stage CPU seconds and calls since the last reset (VisualOdometry.cpp:85-178 stage timers) */
enum { VOO_STAGE_BLUR, VOO_STAGE_RESPONSE, VOO_STAGE_NMS, VOO_STAGE_DESCRIBE, VOO_STAGE_MATCH, VOO_STAGE_RANSAC,
       VOO_STAGE_POSE, VOO_NSTAGES };
void voo_stage_reset(void);
void voo_stage_times(double* seconds, int64_t* calls);
/* gray == NULL: missing image.  gt: 12 doubles (KITTI row) per frame for the whole
 * sequence (gt_n rows) or NULL (scale 1).  pose_out: 12 doubles (3x4 row-major).
 * info_out (optional, 8 ints): n_kpts, n_matches, n_inliers, best_k, n_evaluated, fitted, 0, 0 */
int  voo_vo_process(voo_vo* s, const uint8_t* gray, size_t stride, const double* gt, int gt_n,
                    double pose_out[12], int* status, int32_t* info_out);

#ifdef __cplusplus
}
#endif
#endif
