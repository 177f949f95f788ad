// vo_internal.h -- device-resident state and buffer layout of one vo_ctx, shared by
// the HIP kernels (vo_kernels.hip) and the host driver (vo_api.cpp).
//
// Execution model: frames are processed in WINDOWS of up to B
// frames per launch.  Extract (stencil / select / describe) runs B frames per launch on
// its own queue into a ring of keypoint/descriptor slots; a POSE PASS (match, RANSAC x2,
// refit, triangulate, finalize) runs the window [lo, lo + B) of uncommitted frames, each
// frame speculatively matched against frame f-1.  k_finalize walks the window in frame
// order, applies the trajectory loop's rules (VisualOdometry.cpp:68-189) and commits every
// frame whose speculation holds; the first frame after a skipped one is re-run by the next
// pass against the right previous frame.  So results are those of the sequential loop.
//
// HBM layout (allocated once per ctx in vo_create; the reference allocates every
// cl::Buffer per frame, corner_detection_parallel_GPU.cpp:45-49,85 and
// FREAK_feature_descriptor_parallel_GPU.cpp:53-78).  x B = one copy per frame of a batch.
//   frame_in    u8  W*H            staging for host-supplied frames
//   blurred     u8  Wb*Hb    x B   7x7 Gaussian output (read back by describe); rows of
//                                  Wb >= whole stencil strips + 2, Hb = whole tiles + 4 rows
//   response    f32 W*H            optional dense R map (debug / parity only)
//   cand        u64 232/tile x B   NMS survivors per 57x16 tile, key = Rbits<<32 | row<<16 | col
//   tilerows    u8  16/tile  x B   survivors per tile row (select emits raster order from them)
//   ckeys       u64 232/tile x B   boundary-bin keys of the banded select (single-workgroup
//                                  select: compact survivors when they overflow its LDS)
//   selbits     u64 4/tile   x B   selected-survivor bitmap (only when it overflows LDS)
//   hist        u32 4096     x B   coarse histogram of candidate R (top-N boundary)
//   kps         int2 N  x SLOTS    raster-ordered keypoints: ring slot f % VO_RING, carry, stage
//   desc        u64 8N  x SLOTS    packed 512-test descriptors
//   pre         u32 N   x SLOTS    tests 0..31 (the matcher's 32-bit prefix)
//   match_j     i32 N        x B   best cur index per prev query, -1 if rejected
//   match_pairs int2 N       x B   (prev, cur) matches, ascending prev index
//   pts         f64 4N       x B   matched (x1,y1,x2,y2)
//   pts32       f32 4N       x B   the same in f32, word-swizzled (vo_pts32_index): the Sampson certificate's input
//   hypF        f64 9*H      x B   per-hypothesis F (kept for the refit)
//   counts      i32 H        x B   per-hypothesis inlier counts
//   inlmask     u64 H*N/64   x B   per-hypothesis Sampson inlier bits
//   inl         i32 N        x B   bestInlierSet indices
//   model_p     f32 4N       x B   refit inliers (x1,y1,x2,y2) as cv::Point2f pairs
//   work        VoWork       x B   per-frame control state of the window
//   maxit_tab   u16 tri(N)         ransac.cpp:179-190 iteration bound per (M, best)
//   gt          f64 12*gt_cap      ground-truth rows for the GT scale
//   out         VoFrameOut per frame of a call
#pragma once
#include <stdint.h>

#define VO_HIST_BINS 4096
#ifndef ST_DIAG
#define ST_DIAG 0          // diagnostic build: 1 select archives each frame's key list and per-tile checksums;
                           // 2 + the stencil's own per-tile key / source / response checksums (d.tile_ck, d.dbg 24000..)
#endif
#define VO_DIAG_FRAMES 4096
#define VO_DIAG_KEYS 8192
#ifndef VO_SEL_BANDS
#define VO_SEL_BANDS 8     // select workgroups per frame: bands of tile rows (k_select_count / k_select_emit)
#endif
#ifndef VO_SEL_BANDED_TILES
#define VO_SEL_BANDED_TILES 1024   // banded select for frames of at least this many stencil tiles
#endif
#ifndef VO_TILE_W
#define VO_TILE_W 57       // stencil tile = half a wave's strip x 16 rows (k_stencil ST_TW, ST_TH)
#endif
#define VO_TILE_H 16
#define VO_STRIP_W (2 * VO_TILE_W)   // stencil strip = one wave: two tiles side by side (<= 114: 64 lanes
                                     // of column pairs hold the strip and 7 halo columns each side)
// survivors per tile: strict 3x3 maxima are at most one per 2x2 cell
#define VO_TILE_CAP (((VO_TILE_W + 1) / 2) * ((VO_TILE_H + 1) / 2))
// a stencil lane's first column is xs - VO_STRIP_XL + 2 lane (xs: the strip's first output column)
#define VO_STRIP_XL (128 - VO_STRIP_W - 7 - (128 - VO_STRIP_W - 14) / 2)
// blurred plane column x is stored at byte x + VO_BLUR_X0 of its row, so that the stencil's
// column pairs (even VO_STRIP_XL: even first columns) are 2-byte aligned
#define VO_BLUR_X0 (VO_STRIP_XL & 1)
// blurred plane of a W x H frame: row stride and rows (every stencil wave stores whole rows of
// its strip, up to 4 rows past its segment; a column pair may reach one column past the strips)
inline int vo_blur_stride(int W)
{
    return (((W + VO_STRIP_W - 1) / VO_STRIP_W) * VO_STRIP_W + VO_BLUR_X0 + 1 + 3) & ~3;
}
inline int vo_blur_rows(int H) { return ((H + VO_TILE_H - 1) / VO_TILE_H) * VO_TILE_H + 4; }
// keypoint/descriptor slots: frame f (since vo_reset) is extracted into ring slot
// f % VO_RING; the last valid frame's copy lives in the carry slot during a skip run; the
// stage APIs (vo_extract / vo_match) use their own two slots.  The ring holds d.ring slots
// (VO_RING_DEFAULT = 4096: 0.6 GB at N = 2000, sized for HBM; VO_RING_SLOTS overrides it, the
// tests use small rings to exercise wrap-around)
#define VO_RING_DEFAULT 4096
#define VO_RING (d.ring)
#define VO_CARRY_SLOT (d.ring)
#define VO_STAGE_SLOT (d.ring + 1)
#define VO_SLOTS (d.ring + 3)
// frames per host chunk: a chunk never extracts over a slot one of its passes still reads
// (frame f's slot is rewritten by frame f + VO_RING; passes read frames >= lo - 1)
#define VO_CHUNK (d.ring - 1)
#define VO_MAX_BATCH 128
#ifndef VO_MAX_WIN
#define VO_MAX_WIN 128       // pose window capacity (k_finalize / k_traj LDS; < 255: thread 255 keeps the loop state).
                             // Windows measured: 64 227k, 96 258k, 128 268k, 160 / 192 within noise of 128
#endif
#define VO_MAX_SEQ_STARTS 4096     // vo_set_sequence_starts capacity
#define VO_DEFAULT_BATCH 64
#define VO_REPAIR_WIN_DEFAULT 8   // pose window after a speculation miss (frames; dual records: 4 / 8 / 16 measured 174k / 180k / 177k KITTI frames/s)
#define VO_SLACK_DEFAULT 1        // extra passes per chunk of >= 4 batches (VO_SLACK; 0 / 1 / 4 measured within noise)
// ctr words: cross-queue counters on lines of their own
#ifndef VO_EXT_QUEUES
#define VO_EXT_QUEUES 1        // extract queues and scratch copies: one (two queues, stencil and select + describe
                               // split over them, queue priorities and paired stencil launches were measured and
                               // removed in round 6: none was faster, each multiplied the cross-queue orderings)
#endif
#define VO_CTR_DESCRIBE 0      // + 16 * queue: describe's in-launch arrival counter
#define VO_SYNC_EXT 32         // + 16 * queue: frames extracted since vo_reset by that queue
                               // (its batches complete in order; the pose queue waits on it)
#define VO_CTR_FIN 64          // fused triangulate + finalize: workgroups arrived (the last one finalizes)
#define VO_CTR_ERR 80          // device consistency failures (k_select / k_select_count: VO_STATUS_INCONSISTENT)
#define VO_CTR_WORDS 96
// host-frame streaming (vo_process_frames_host): device ring of VO_HRING slots of B frames
#define VO_HRING 3
#define VO_HOST_FIRST_BATCH 16 // host streaming: frames in a chunk's first batch (shorter pipeline fill)
#define VO_EV_WAIT 0           // per-batch event pools of a chunk (vo_api.cpp)
#define VO_EV_COPY 1
#define VO_EV_STENCIL 2
#define VO_EV_SPLIT_S 3        // split extract: stencil of batch j done (select / describe queue waits)
#define VO_EV_SPLIT_D 4        // split extract: describe of batch j done (its scratch copy is free again)
#define VO_EV_POOLS 5
#define VO_MAX_HYP 2000
#ifndef VO_RESP_SCALE
// The stencil computes twice the corner response, tr - sqrt(tr^2 - 4 det), without the reference's
// final halving (kernel .c:108-114: (tr * 0.5) - (0.5 * s), which is exactly half of it): every
// consumer only orders responses or compares them with the threshold, and doubling is exact and
// order-preserving (the threshold is doubled with them, d.resp_thr; the select's histogram bins,
// (bits - thr_bits) >> 15, are unchanged since both exponents grow by one).  The response map
// (vo_response) is halved back.  Two VALU fewer per stencil row.
#define VO_RESP_SCALE 2
#endif
#define VO_HYP_CHUNK0 100     // RANSAC launch chunks (vo_kernels.hip launch_ransac); 100 = the clamp
#define VO_HYP_CHUNK1 700     // the later chunks [100, 700) and [700, 2000) (VO_HYP_CUTS): most frames' adaptive loops stop before 700, and the second chunk's replay lets their [700, 2000) exit at once
#define VO_HYP_REPS 1        // hypotheses per wave in the last chunk (VO_RREPS; 4 and 8 measured 1-6 % slower)

struct VoFrameOut {
    int32_t status, n_kps, n_matches, n_inl, best_k, n_eval, fitted, frame;
    int32_t err;          // the frame's extract failed the select's consistency check (VO_STATUS_INCONSISTENT;
                          // reported even where the status is FIRST): the call returns VO_ERR_INTERNAL
    int32_t pad;
    double pose[12];
};


// Per-frame control state of a pose pass (one per window frame).  k_match writes the
// header, the RANSAC launches their counters and the replay's result, k_refit the model,
// k_triangulate the cheirality counts; k_finalize reads it all.
struct VoWork {
    int32_t status;       // VO_STATUS_* (speculative: assumes frame - 1 was a valid frame)
    int32_t frame;        // frame index since vo_reset
    int32_t cur, prev;    // keypoint/descriptor slots
    int32_t M;            // matches
    int32_t scored;       // T * floor(M / T)   (ransac.cpp:152-157)
    int32_t maxit, best, bestk, k_done, need_more, n_eval;
    int32_t n_inl;        // best hypothesis' inlier count
    int32_t fitted;       // refit ran (>= 8 inliers); else the model leaks (quirk 9)
    int32_t n_fit;        // refit inliers (== n_inl when fitted)
    int32_t degenerate;   // getPose would throw on this frame's F (PoseUpdate.hpp:71-73)
    int32_t nv_status;    // refit null-vector solver: 0 converged, 1 certified after the cap, 2 Jacobi fallback
    int32_t cold;         // refit from x0 = ones instead of the best hypothesis (vo_fit_F, stage only)
    int32_t counts4[4];   // positive-depth counts per (R, t) candidate
    uint32_t ctr[4];      // in-launch arrival counters: [0] match, [1] ransac chunk 1, [2] chunk 2
    uint32_t ready1;      // k_ransac_fused: the first chunk's replay is written (reset by k_match's header)
    uint32_t pad1;
    uint64_t frame_seed;
    float cmax[4];        // bounds of |x|, |y|, |x'|, |y'| over the scored matches (the f32 Sampson
                          // certificate's magnitudes, vo_sampson32.h): W, H, W, H for a pose pass
    double F[9];          // refit F (valid iff fitted)
    double R1[9], R2[9], t[3];
};

// A committed frame's input to the trajectory (written by k_finalize, read by k_traj on the
// trajectory queue): the relative motion's model (R, unit t before the GT scale) and the
// frame's kind.  Ring of d.ring records, frame f at f % ring.
struct VoTrajRec {
    double R[9], t[3];
    int32_t kind;         // 1: T_curr = T_curr * T_rel (a posed frame); 0: T_curr unchanged
    int32_t first;        // FIRST: T_curr = eye(4) (VisualOdometry.cpp:57)
    int32_t flip;         // the row is flipZ * T_curr (all but FIRST / MISSING)
    int32_t lvb;          // last valid frame before it (the GT scale's reference)
};
#define VO_PLOG 4096       // pass log ring: (lo, committed frames) of pass p at p % VO_PLOG

// Cross-pass pipelining: a pass's match and RANSAC run on the pose queue
// while the previous pass's refit, triangulation and finalize run on the fit queue, so pass p
// chooses its window before pass p - 1 has committed.  k_match decides it from the state after
// pass p - 2 (its snapshot; the pose queue waited for that finalize) and pass p - 1's window:
// if pass p - 1 starts where pass p - 2 left the trajectory (its window start and first-frame
// desc1 slot), pass p speculates that p - 1 commits its whole window and starts after it;
// otherwise pass p - 1 will be discarded and pass p starts from the snapshot.  k_finalize commits
// a pass only if its window start and first-frame desc1 slot match the trajectory state then
// (a speculation miss discards it; the next pass restarts from the state).  Rings of 4 by pass.
#define VO_PASS_RING 4
struct VoPlan {           // the window of pose pass p (k_match's first workgroup writes it)
    int32_t lo, n;        // frames [lo, lo + n)
    int32_t dual;         // a repair window with two work records per frame
    int32_t prev0;        // desc1 slot the window's first frame was matched against
};
struct VoSnap {           // the trajectory state after pass p's k_finalize
    int32_t lo, prev_slot, win, dual;
};

// Trajectory state (VisualOdometry::run's locals), read and written by k_finalize only
// (T_curr: by k_traj only).
struct VoState {
    int32_t lo;           // frames committed since vo_reset (the next pass starts here)
    int32_t end;          // unused (a pass's window is bounded by d.gmax, <= the frames enqueued)
    int32_t prev_slot;    // slot of the last valid frame's keypoints / descriptors (desc1)
    int32_t last_valid;   // VisualOdometry.cpp:62,164
    int32_t model_n;      // FundamentalMatrix model (VisualOdometry.cpp:49): inliers of the last fit
    int32_t model_degenerate;
    int32_t pose_status;  // stage vo_pose result
    int32_t win;          // frames in the next pass's window: B, or repair_win after a pass that stopped early
    int32_t dual;         // the next pass is a repair window: each frame also matched against desc1 (prev_slot)
    int32_t pad;
    double model_F[9];
    double model_R[9], model_t[3];   // getPose(model) before scaling: det-fixed R, signed unit t
    double Tcurr[16];
    double pose_R[9], pose_t[3];     // stage vo_pose result
    double scale_override;           // stage vo_pose scale
};

// Banded select's per-frame hand-off (x B x VO_EXT_QUEUES): k_select_count's workgroups publish
// their band's count above the boundary bin and append the boundary bin's keys; the last one to
// arrive ranks the boundary keys and writes the threshold and each band's first output position
// for k_select_emit (the kernel boundary orders them).
struct VoSelCtl {
    uint32_t arrive;                 // workgroups of the frame arrived (reset by the last)
    uint32_t nbnd;                   // boundary-bin keys appended (reset by the last)
    int32_t dcount[VO_SEL_BANDS];    // per band: keys above the boundary bin
    int32_t b;                       // boundary bin, -1: every key is selected
    int32_t pad;
    uint64_t Tb;                     // smallest selected key of the boundary bin
    int32_t base[VO_SEL_BANDS];      // per band: its first keypoint position in raster order
    int32_t ktot[VO_SEL_BANDS];      // per band: its keys by the stencil's tile row counts (the
                                     // consistency check: their sum must equal the histogram's total)
    uint32_t ready;                  // k_select_fused: the threshold and band positions are written
    uint32_t arrive2;                // k_select_fused: bands done emitting (the last clears ready)
    uint32_t timeout;                // k_select_fused: a band timed out waiting for ready (the last band
                                     // to finish emitting marks the slot INCONSISTENT after the ranker's
                                     // OK store, then clears it)
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
    int max_hyp;
    int B;                // extract batch capacity (frames)
    int WB;               // pose window capacity (frames): min(2 B, VO_MAX_WIN), VO_WIN overrides
    int gridw;            // window records a pose-pass launch covers (blockIdx.y): WB; 2 for the single-frame call
    int single;           // the single-frame call (vo_process_frame): latency-shaped launches
    int gmax;             // pose pass: frames < gmax are extracted (the pass's wait covers them)
    int eq;               // extract queue of this launch (its scratch copy and counters)
    int xcd_map;          // extract kernels place a frame's workgroups on one XCD (VO_XCD=0: off)
    int repair_win;       // window after a pass whose commit stopped early (VO_REPAIR_WIN, default VO_REPAIR_WIN_DEFAULT)
    uint64_t seed;
    double K[9];
    uint32_t cand_cap;    // per frame
    int ntiles;
    int gt_n;
    uint8_t* frame_in;
    uint8_t* blurred;     // x B: bplane bytes per frame, rows of bstride
    int bstride;
    size_t bplane;
    float* response;
    uint64_t* cand;       // x B: per stencil tile up to 192 keys in tile-local raster order
    uint8_t* tilerows;    // x B: per stencil tile the candidate count of each of its 16 rows
    uint64_t* ckeys;      // x B: select's compact keys when they exceed the LDS capacity
    uint64_t* selbits;    // x B: select's selected-key bitmap when it exceeds the LDS capacity
    int sel_lds;          // select (single-workgroup form, VO_SEL1=1): dynamic LDS bytes
    int sel_emit_lds;     // banded select: k_select_emit's dynamic LDS bytes (a band's segment counts)
    int sel1;             // VO_SEL1=1: the single-workgroup select (one 1024-thread workgroup per frame)
    int sel_fused;        // the per-frame call's banded select in one launch (k_select_fused; VO_SEL_FUSED=0: two);
                          // 2: keys staged in LDS, the bitmap built before the wait (VO_SEL_EARLY=0: 1)
    int ransac_fused;     // one frame's two RANSAC chunks in one launch (k_ransac_fused; VO_RANSAC_FUSED=0: two)
    int rng_mode;         // VO_RNG_MT19937: the hypotheses' samples come from `samples` (host-drawn std::sample)
    int32_t* samples;     // x WB records: max_hyp x 8 indices per record (VO_RNG_MT19937 only)
    VoSelCtl* selctl;     // x B x VO_EXT_QUEUES
    uint32_t* hist;       // x B (scratch of extract queue eq; x VO_EXT_QUEUES allocated)
    int2* kps;            // x SLOTS (N each)
    uint64_t* desc;       // x SLOTS (8N each)
    uint32_t* pre;        // x SLOTS (N each)
    int32_t* match_j;     // x B
    int2* match_pairs;    // x B
    double* pts;          // x B
    float* pts32;         // x B: the same points in f32, per 64-match word [component][j / 4][r][j % 4]
                          // (match 64 w + 8 j + r; vo_pts32_index), for the f32 Sampson certificate
    double* hypF;         // x B
    int32_t* counts;      // x B
    int32_t* inl;         // x B
    uint64_t* inlmask;    // x B: per hypothesis the Sampson inlier bits of the scored matches
    int mask_words;       // (N + 63) / 64
    float* model_p;       // x B
    VoWork* work;         // x B
    const uint16_t* maxit_tab;
    const double* gt;
    VoState* st;
    int ring;             // ring slots (VO_RING)
    int32_t* ext_n;       // x SLOTS: keypoints extracted into the slot
    int32_t* ext_st;      // x SLOTS: VO_STATUS_OK, VO_STATUS_OVERFLOW (select capacity), VO_STATUS_MISSING,
                          // VO_STATUS_INCONSISTENT (the select's consistency check failed; ctr[VO_CTR_ERR] counts them)
    const int32_t* seq_starts;   // sorted frame indices (since vo_reset) where a new sequence begins
    int n_seq_starts;
    int origin;           // in-sequence index of frame 0 of the stream's first sequence (a shard of one sequence)
    unsigned* ctr;
    VoTrajRec* trec;      // x ring: committed frames' trajectory inputs (k_finalize -> k_traj)
    int2* plog;           // x VO_PLOG: (lo, committed) per pose pass
    int32_t* lo_host_dev; // pinned host word (device address): each k_traj stores VoState::lo there (the commit point)
    int pass;             // pose pass number (its plog entry)
    int nospec;           // every earlier pass is finalized: the window comes from the state itself
    VoPlan* plan;         // x VO_PASS_RING
    VoSnap* snap;         // x VO_PASS_RING
    unsigned long long* dbg;   // diagnostic s_memtime stamps (VO_STAMPS builds only)
    unsigned long long* tile_ck;   // ST_DIAG builds: x B x VO_EXT_QUEUES, per tile the stencil's key checksum
    // ST_DIAG builds, per frame f < VO_DIAG_FRAMES of the call (frame index since vo_reset):
    unsigned long long* diag_tile;   // [f][tile]  select: checksum of the tile's keys as read
    unsigned long long* diag_src;    // [f][tile]  stencil: checksum of the source rows a wave consumed (even tiles)
    unsigned long long* diag_resp;   // [f][tile]  stencil: checksum of the responses a wave computed (even tiles)
    unsigned long long* diag_keys;   // [f][VO_DIAG_KEYS] select: the frame's compact key list (first VO_DIAG_KEYS)
    int diag_f0;                     // frame index of batch frame 0 (enqueue_extract)
    int fault_inject;                // VO_FAULT_INJECT=1 (tests only): launch_stencil adds N counts to each frame's
                                     // top histogram bin, so the select's consistency check must fire
    unsigned spin_limit;             // polls of the fused select's / fused RANSAC's bounded waits (1 << 22;
                                     // VO_SPIN_LIMIT=0, tests only: every wait times out at once)
};

// launch wrappers (vo_kernels.hip)
#include <hip/hip_runtime.h>
// f32 copy of match i's component c (0..3: x, y, x', y') in a frame's pts32 block: lane r of the
// RANSAC count's lane groups reads components of its matches 64 w + 8 j + r, j = 4 q .. 4 q + 3, as
// one float4 (vo_kernels.hip count_words32)
__host__ __device__ inline size_t vo_pts32_index(int i, int c)
{
    const int w = i >> 6, j = (i >> 3) & 7, r = i & 7;
    return (size_t)w * 256 + (size_t)c * 64 + (size_t)(j >> 2) * 32 + (size_t)r * 4 + (size_t)(j & 3);
}
// pts32 entries per frame record: whole words
#define VO_PTS32_PER(N) ((size_t)(((N) + 63) / 64) * 256)

namespace vo {
// extract of nb frames: frame f0 + z reads img0 + z * frame_bytes into slot
// (slot_override >= 0 ? slot_override : (f0 + z) % VO_RING), scratch z.  publish > 0: the
// last describe workgroup stores it to ctr[VO_SYNC_EXT] for the pose queue
void launch_stencil(const VoDev& d, const uint8_t* img0, size_t frame_bytes, int nb, int write_response, hipStream_t s);
void launch_select(const VoDev& d, int f0, int nb, int slot_override, hipStream_t s);
int select_lds_bytes(int W, int H, int* key_cap);     // sets the kernel attribute; <0 on failure
int select_emit_lds_bytes(int W, int H);              // banded select: sets the attribute; <0 if the band does not fit
int select_fused_lds_bytes(int W, int H);             // k_select_fused with staged keys: sets the attribute; <0: no fit
void launch_describe(const VoDev& d, int f0, int nb, int slot_override, unsigned publish, hipStream_t s);
void launch_ext_missing(const VoDev& d, int slot, hipStream_t s);   // extract side of a missing image
// the pose queue's wait for an extract batch (VO_EVENT_WAIT=0): one wave polls ctr[VO_SYNC_EXT]
// until describe has published `target` frames
void launch_wait_ext(const VoDev& d, unsigned target, hipStream_t s);
// pose pass over the window (stage = 0) or over work[0] prepared by a stage API (stage = 1)
void launch_match(const VoDev& d, int stage, hipStream_t s);        // + ordered compaction per frame
void launch_ransac(const VoDev& d, int stage, hipStream_t s, int part = 0);   // all hypotheses + replay per frame
// (part 1: only the first chunk [0, VO_HYP_CHUNK0) and its replay; part 2: only the later chunks)
void launch_refit(const VoDev& d, int with_pose, int stage, hipStream_t s);
// fin: the pass's finalize in the last workgroup of the launch (out / out_base as launch_finalize)
void launch_triangulate(const VoDev& d, int stage, hipStream_t s, VoFrameOut* out = nullptr, int out_base = 0, int fin = 0);
void launch_finalize(const VoDev& d, VoFrameOut* out, int out_base, hipStream_t s);
void launch_traj(const VoDev& d, VoFrameOut* out, int out_base, hipStream_t s);   // T_curr chain + pose rows of pass d.pass
void launch_traj_range(const VoDev& d, VoFrameOut* out, int out_base, int lo, int nc, hipStream_t s);   // vo_rechain
void launch_pose_stage(const VoDev& d, int phase, hipStream_t s);   // vo_pose: 0 prepare, 1 choose
void launch_reset(const VoDev& d, hipStream_t s);                   // vo_reset's device state
// n bytes from pinned host memory to the device by a copy kernel on s (a single frame's upload:
// no copy-engine -> compute-queue hand-off in front of the stencil)
void launch_h2d(uint8_t* dst, const uint8_t* src_pinned, size_t n, hipStream_t s);
void launch_selftest_nullvec9(const double* S, const double* x0, double* f, int* status, int n, hipStream_t s);
void launch_selftest_arith(const float* fa, const float* fb, float* fo, const double* da,
                           const double* db, double* dout, int n, hipStream_t s);
int kernel_count();
const char* kernel_form(const VoDev& d, int k);   // the kernel symbol(s) stage k launches (profiles)
const char* kernel_name(int i);
}  // namespace vo
