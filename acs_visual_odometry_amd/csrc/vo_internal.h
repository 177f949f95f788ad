// vo_internal.h -- device-resident state and buffer layout of one vo_ctx, shared by
// the HIP kernels (vo_kernels.hip) and the host driver (vo_api.cpp).
//
// HBM layout (allocated once per ctx in vo_create; the reference allocates every
// cl::Buffer per frame, corner_detection_parallel_GPU.cpp:45-49,85 and
// FREAK_feature_descriptor_parallel_GPU.cpp:53-78):
//   frame_in    u8  W*H         staging for host-supplied frames
//   blurred     u8  W*H         7x7 Gaussian output (read back by describe)
//   response    f32 W*H         optional dense R map (debug / parity only)
//   cand        u64 256/tile    NMS survivors per 64x16 tile, key = Rbits<<32 | row<<16 | col
//   tilerows    u8  16/tile     survivors per tile row (select emits raster order from them)
//   ckeys       u64 256/tile    compact survivors (only when they overflow select's LDS)
//   selbits     u64 4/tile      selected-survivor bitmap (only when it overflows LDS)
//   hist        u32 4096        coarse histogram of candidate R (top-N boundary)
//   kps[2]      int2 N          raster-ordered keypoints, slot ping-pong
//   desc[2]     u64 8N          packed 512-test descriptors (slot ping-pong)
//   pre[2]      u32 N           tests 0..31 (the matcher's 32-bit prefix)
//   match_j     i32 N           best cur index per prev query, -1 if rejected
//   pts         f64 4N          matched (x1,y1,x2,y2), ascending prev index
//   hypF        f64 9*2000      per-hypothesis F (kept for the refit)
//   counts      i32 2000        per-hypothesis inlier counts
//   inl         i32 N           bestInlierSet indices
//   model_p     f32 4N          model inliers (x1,y1,x2,y2) as cv::Point2f pairs
//   maxit_tab   u16 tri(N)      ransac.cpp:179-190 iteration bound per (M, best)
//   gt          f64 12*gt_cap   ground-truth rows for the GT scale
//   out         VoFrameOut per frame of a batch
#pragma once
#include <stdint.h>

#define VO_HIST_BINS 4096
// keypoint/descriptor slots: frame f of the pipeline extracts into ring slot f % VO_RING_SLOTS;
// a prev that must outlive its ring slot (frames skipped after it) is copied to the carry
// slot; the stage APIs (vo_extract / vo_match) use their own two slots
#define VO_RING_SLOTS 8
#define VO_CARRY_SLOT 8
#define VO_STAGE_SLOT 9
#define VO_SLOTS 11
#define VO_EXT_RING 16         // per-frame extract results, indexed f & (VO_EXT_RING - 1)
#define VO_EXT_QUEUES 3        // extract queues: frame f on queue f % VO_EXT_QUEUES (+1 pose queue = 4 HW queues)
// ctr words: in-launch arrival counters [0, VO_CTR_COUNTERS), then the cross-queue frame
// counters on lines of their own: the pose chain's (monotonic, read by the extract queues'
// stream-wait-value packets) and one extract-done word per ring entry (polled by k_match)
#define VO_CTR_COUNTERS 16
#define VO_CTR_DESCRIBE 4      // + extract queue
#define VO_SYNC_POSE 48        // frames whose pose chain is complete
#define VO_SYNC_EXT 64         // + (f & (VO_EXT_RING - 1)): f + 1 once frame f is extracted
#define VO_CTR_WORDS 96
#define VO_MAX_HYP 2000
#define VO_HYP_CHUNK0 256
#define VO_RED_THREADS 256

// frame modes for k_frame_begin
#define VO_MODE_FRAME 0        // full trajectory-loop iteration
#define VO_MODE_MISSING 1      // image missing: only push T_curr
#define VO_MODE_EXTRACT 2      // vo_extract: extract into slot 0, no state change
#define VO_MODE_STAGE 3        // stage APIs (match / ransac / pose): status OK, no trajectory

struct VoFrameOut {
    int32_t status, n_kps, n_matches, n_inl, best_k, n_eval, fitted, frame;
    double pose[12];
};

// Extract-side state.  The extract kernels of frames f+1, f+2, ... run on their own queues
// while frame f's match -> pose chain runs; they never touch VoState, and the pose chain only
// reads the ring entries of its own frame here (the carry copy in finalize reads a slot no
// extract in flight writes), so the queues never write the same field.
struct VoExt {
    int32_t slot[VO_EXT_RING];    // slot extracted for frame f (ring f & 15); -1: image missing
    int32_t status[VO_EXT_RING];  // VO_STATUS_OK, or VO_STATUS_OVERFLOW (select capacity)
    int32_t n_kps[VO_SLOTS];
    int32_t stage_status;  // status of the last stage extract (vo_extract)
    int32_t pad[2];
};

struct VoState {
    int32_t frame;        // index of the frame being processed
    int32_t status;       // VO_STATUS_* of the current frame
    int32_t mode;
    int32_t cur, prev;    // keypoint/descriptor slots: prev always; cur only in stage mode
                          // (frame mode: VoExt::slot[frame & (VO_EXT_RING - 1)])
    uint32_t cand_count;
    int32_t M;            // matches
    int32_t scored;       // T * floor(M / T)   (ransac.cpp:152-157)
    int32_t maxit, best, bestk, k_done, need_more, n_eval;
    int32_t n_inl, fitted;
    int32_t model_n;
    int32_t degenerate;
    int32_t counts4[4];
    int32_t last_valid;
    int32_t out_index;    // slot in the batch output array
    int32_t pad0;
    uint64_t frame_seed;
    double model_F[9];
    double R1[9], R2[9], t[3];
    double pose_R[9], pose_t[3];   // last getPose result (stage API)
    double scale_override;         // NaN: GT-derived scale
    double Tcurr[16];
};

// Everything a kernel needs, passed by value.
struct VoDev {
    int W, H, N;
    int nms_k, brow, bcol;
    float resp_thr;
    uint32_t thr_bits;
    float ratio;
    int match_bits;
    double ransac_p, sampson_thr;
    int T;
    int maxit_initial;
    uint64_t seed;
    double K[9];
    uint32_t cand_cap;
    int gt_n;
    uint8_t* frame_in;
    uint8_t* blurred;
    float* response;
    uint64_t* cand;       // per stencil tile: up to 256 keys in tile-local raster order
    uint8_t* tilerows;    // per stencil tile: candidate count of each of its 16 rows
    uint64_t* ckeys;      // select: compact candidate keys when they exceed the LDS capacity
    uint64_t* selbits;    // select: selected-key bitmap when it exceeds the LDS capacity
    int sel_lds;          // select: dynamic LDS bytes
    uint32_t* hist;
    int2* kps[VO_SLOTS];
    uint64_t* desc[VO_SLOTS];
    uint32_t* pre[VO_SLOTS];
    int32_t* match_j;
    int2* match_pairs;
    double* pts;
    double* hypF;
    int32_t* counts;
    int32_t* inl;
    uint64_t* inlmask;    // per hypothesis: Sampson inlier bits of the scored matches
    int mask_words;       // (N + 63) / 64
    float* model_p;
    const uint16_t* maxit_tab;
    const double* gt;
    VoState* st;
    VoExt* ext;
    VoFrameOut* out;
    unsigned* ctr;        // in-launch arrival counters: [0] match, [1] ransac, [2] triangulate,
                          // [3] ransac chunk 2, [4] describe; cross-queue counters (VO_SYNC_*)
    uint32_t seqno;       // frame pipeline: 1 + frame index since vo_reset; 0 outside it
    uint32_t wait_next;   // finalize then waits for this frame's extract (seqno + 1), or 0
    int eq;               // extract queue of this frame (its scratch: blurred .. hist)
    unsigned long long* dbg;   // diagnostic s_memtime stamps (VO_STAMPS builds only)
};

// launch wrappers (vo_kernels.hip)
#include <hip/hip_runtime.h>
namespace vo {
void launch_frame_begin(const VoDev& d, int mode, hipStream_t s);
void launch_stencil(const VoDev& d, const uint8_t* frame, int write_response, hipStream_t s);
// fidx: frame index since vo_reset (frame pipeline; select picks the slot), or -1 for the
// stage API (slot VO_STAGE_SLOT)
void launch_select(const VoDev& d, int fidx, hipStream_t s);
int select_lds_bytes(int W, int H, int* key_cap);     // sets the kernel attribute; <0 on failure
void launch_describe(const VoDev& d, int fidx, hipStream_t s);
void launch_ext_missing(const VoDev& d, int fidx, hipStream_t s);   // extract side of a missing image
void launch_match(const VoDev& d, hipStream_t s);          // + ordered compaction (last workgroup)
void launch_ransac(const VoDev& d, int nhyp, hipStream_t s); // all hypotheses + replay (last workgroup)
void launch_refit(const VoDev& d, int with_pose, hipStream_t s);
void launch_pose_prep(const VoDev& d, hipStream_t s);
void launch_triangulate(const VoDev& d, hipStream_t s);    // + finalize / next-frame setup
void launch_missing(const VoDev& d, hipStream_t s);
void launch_selftest_arith(const float* fa, const float* fb, float* fo, const double* da,
                           const double* db, double* dout, int n, hipStream_t s);
int kernel_count();
const char* kernel_name(int i);
}  // namespace vo
