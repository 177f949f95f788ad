// vo_api.cpp -- host side of libvo_mi355x.so: the C ABI of include/vo_mi355x.h.
//
// One vo_ctx = one GPU + two HIP streams + every device buffer of the path allocated
// once (HBM layout: vo_internal.h).  Per frame the host only enqueues kernels; all
// per-frame decisions of the reference's trajectory loop (skip on < 8 matches /
// inliers, descriptor carry-forward, RANSAC model leak, GT scale) are taken on the
// device from VoState, so frames can be enqueued back to back with no host sync.
//
// Frame pipeline (vo_process_frames_device): frames are extracted B per launch on stream
// `se` into a ring of VO_RING keypoint/descriptor slots; pose passes on stream `s` each take
// the window of the next B uncommitted frames (match, RANSAC, refit, triangulate: one
// launch each for the whole window; finalize commits in frame order, vo_internal.h).  The
// pose queue waits for each extract batch on its event (or a polling wait kernel); a chunk of at
// most VO_CHUNK frames never rewrites a slot its passes still read, so the extract queue
// runs ahead freely.  One host sync per chunk reads how far the passes committed.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <climits>
#include <map>
#include <memory>
#include <iterator>
#include <mutex>
#include <new>
#include <numeric>
#include <random>
#include <utility>
#include <vector>

#include "vo_internal.h"
#include "../../include/vo_mi355x.h"


struct vo_ctx {
    vo_config cfg;
    VoDev d;
    hipStream_t s = nullptr;          // pose passes, stage APIs, the single-frame path
    hipStream_t se[VO_EXT_QUEUES] = {};   // the extract queue of the device path (se[0])
    int B = VO_DEFAULT_BATCH;         // frames per extract batch / pose-pass window
    int Bx = VO_DEFAULT_BATCH;        // extract batch capacity: B + B / 2 (a chunk's short tail joins its last batch)
    int fidx = 0;                     // frames enqueued since vo_reset
    int mt_err = 0;                   // VO_RNG_MT19937: a failed sample upload of a pass (returned by run_chunk)
    bool serial = false;              // VO_SERIAL=1: every kernel on one queue, no cross-queue
                                      // waits (for profilers that serialize dispatches: PMC passes)
    bool event_wait = true;           // pose queue waits for extract batches on events, or (VO_EVENT_WAIT=0)
                                      // in a one-wave kernel polling the counter describe publishes
    int slack = 0;                    // VO_SLACK: extra passes enqueued per chunk (misses re-run without a host round trip)
    hipStream_t st = nullptr;         // trajectory queue: k_traj of each pass (T_curr chain, pose rows)
    hipEvent_t ev_fin = nullptr;      // a pass's k_finalize done (the trajectory queue waits on it)
    hipStream_t sf = nullptr;         // fit queue: refit, triangulation and finalize of pipelined passes
    static constexpr int kPassEv = 8;
    hipEvent_t ev_rs[kPassEv] = {};   // pass p's RANSAC done (the fit queue waits on it), p % 8
    hipEvent_t ev_fn[kPassEv] = {};   // pass p's finalize done (pass p + 2 and the trajectory queue wait on it)
    hipEvent_t ev_r2[kPassEv] = {};   // pass p's later RANSAC chunks done (rq: the fit queue waits on it)
    bool rq = false;                  // later RANSAC chunks on the trajectory queue, k_traj on the fit queue
    bool pipeline = true;             // VO_PIPELINE=0: every pass on the pose queue, one after the other
    size_t set_off[10] = {};           // element offsets of window buffer set 1 (pass p uses set p & 1)
    int npass = 0;                    // pose passes enqueued (their pass-log entries)
    // per-batch event pools of a chunk: [VO_EV_WAIT] extract done (event_wait mode),
    // [VO_EV_COPY] H2D copy done, [VO_EV_STENCIL] stencil done (host streaming)
    std::vector<hipEvent_t> ev_batch[VO_EV_POOLS];
    hipStream_t sc = nullptr;         // host streaming: H2D copies of frame batches
    uint8_t* dring = nullptr;         // host streaming: VO_HRING device slots of B frames
    uint8_t* hstage = nullptr;        // host streaming: pinned staging ring for pageable sources
    int gt_cap = 0;
    // GT rows [0] and sequence starts [1]: pinned staging of their asynchronous uploads (upload_meta)
    void* meta_host[2] = {};
    size_t meta_cap[2] = {};
    hipEvent_t ev_meta[2] = {};                       // the last upload from each staging buffer
    hipEvent_t ev_meta_q[VO_EXT_QUEUES + 2] = {};     // the other queues' work before an upload
    VoFrameOut* out_dev = nullptr;
    int out_cap = 0;
    VoFrameOut* out_host = nullptr;   // pinned
    VoFrameOut* out_host_dev = nullptr;   // out_host as the device addresses it (the per-frame call's kernels
                                          // write its row there directly: no copy kernel behind the pass)
    int32_t* lo_host = nullptr;       // pinned: VoState::lo after a chunk
    hipEvent_t ev_reset = nullptr;    // recorded on s by vo_reset; the extract queue waits on it
    bool reset_pending = false;
    uint8_t* stage_host = nullptr;    // pinned frame staging
    uint16_t* tab_dev = nullptr;
    double stage_F[9] = {0};          // vo_ransac_F's FundamentalMatrix (persists across calls)
    std::map<double, uint16_t*> tab_by_p;   // vo_ransac_run: the maxIterations table of the last other probability
    int timing = 0;                   // 0 off, 1 all kernels, 100+k only kernel k
    std::vector<hipEvent_t> ev_pool;
    std::vector<float> ktime_ms;
    std::vector<int> kcount;          // timed launches per kernel
    std::vector<int> klaunch;         // launches per kernel in the last call
    int last_frames = 0;
    // VO_PF_PROFILE=1: host-side phases of vo_process_frame (us, summed; printed by vo_destroy)
    bool pf_profile = false;
    // VO_HOST_PROFILE=1: host time of each run_frames call to its first extract launch, its last pass
    // launch and its return (stderr)
    bool host_profile = false;
    // work may be in flight on the extract, fit or trajectory queues (set when a call enqueues there,
    // cleared once that call has synchronised them all): upload_meta orders its copy after them only then
    bool others_busy = true;
    bool out_zc = true;               // VO_OUT_ZC: batched calls write their rows and commit point to pinned host memory
    std::vector<float> kcont_ms;      // per kernel: the continuation spans' share of ktime_ms (other queues)
    double hp_t[3] = {0.0, 0.0, 0.0};
    double pf_t[5] = {0, 0, 0, 0, 0};     // sync, copy, enqueue, wait, total
    long pf_n = 0;
    double pf_enq_end = 0, pf_wait_end = 0;
    struct Buf { const char* name; uint64_t ptr, bytes; };
    std::vector<Buf> layout;          // device buffers allocated by vo_create (vo_debug_layout)
};

namespace {

int hip_ok(hipError_t e)
{
    if (e != hipSuccess) {
        fprintf(stderr, "[vo_mi355x] HIP error %d: %s\n", (int)e, hipGetErrorString(e));
        return VO_ERR_HIP;
    }
    return VO_OK;
}
#define HIPCHK(x)                          \
    do {                                   \
        int _rc = hip_ok(x);               \
        if (_rc != VO_OK) return _rc;      \
    } while (0)

// ransac.cpp:131 -- double -> int as compiled on x86 (cvttsd2si), see oracle to_int_x86
int to_int_x86(double q)
{
    if (!(q > -2147483649.0 && q < 2147483648.0)) return INT_MIN;
    return (int)q;
}

// maxIterations after a strictly better count (ransac.cpp:179-190), evaluated with the
// host libm exactly as the reference evaluates it; 0xFFFF = "denom == 0: no update".
// Table row M holds entries best = 0..M at offset M(M+1)/2.
// Bounded: at most VO_TAB_CACHE tables (a caller cycling through probabilities would otherwise grow
// host memory without bound, ~17 MB per table at N = 4096); callers hold a shared_ptr while they use one.
#define VO_TAB_CACHE 4
std::mutex g_tab_mu;
std::vector<std::pair<std::pair<int, double>, std::shared_ptr<const std::vector<uint16_t>>>> g_tab_cache;

std::shared_ptr<const std::vector<uint16_t>> maxit_table(int N, double prob)
{
    const auto key = std::make_pair(N, prob);
    {
        std::lock_guard<std::mutex> lk(g_tab_mu);
        for (const auto& e : g_tab_cache)
            if (e.first == key) return e.second;
    }
    auto tab = std::make_shared<std::vector<uint16_t>>((size_t)(N + 1) * (N + 2) / 2, 0xFFFFu);
    const double lp = std::log(1.0 - prob);
    for (int M = 8; M <= N; ++M) {
        uint16_t* row = tab->data() + (size_t)M * (M + 1) / 2;
        for (int best = 1; best <= M; ++best) {
            double outlierRatio = 1.0 - (double)best / (double)M;
            double denom = std::log(1.0 - std::pow(1.0 - outlierRatio, 8.0));
            if (denom == 0.0) { row[best] = 0xFFFFu; continue; }
            int v = to_int_x86(lp / denom);
            v = std::min(std::max(v, 100), 2000);
            row[best] = (uint16_t)v;
        }
    }
    std::lock_guard<std::mutex> lk(g_tab_mu);
    if (g_tab_cache.size() >= VO_TAB_CACHE) g_tab_cache.erase(g_tab_cache.begin());   // the oldest
    g_tab_cache.emplace_back(key, tab);
    return tab;
}

template <typename T>
int dalloc(T** p, size_t n)
{
    return hip_ok(hipMalloc((void**)p, std::max<size_t>(n, 1) * sizeof(T)));
}
// dalloc of a context buffer, recorded for vo_debug_layout (which buffer an address falls in)
template <typename T>
int dalloc_rec(vo_ctx* c, const char* name, T** p, size_t n)
{
    const int rc = dalloc(p, n);
    if (rc == VO_OK) c->layout.push_back({name, (uint64_t)(uintptr_t)*p, (uint64_t)(std::max<size_t>(n, 1) * sizeof(T))});
    return rc;
}

int sync_all(vo_ctx* c)
{
    for (hipStream_t q : c->se)
        if (q) HIPCHK(hipStreamSynchronize(q));
    if (c->s) HIPCHK(hipStreamSynchronize(c->s));
    if (c->sf) HIPCHK(hipStreamSynchronize(c->sf));
    if (c->st) HIPCHK(hipStreamSynchronize(c->st));
    c->others_busy = false;
    return VO_OK;
}
#define SYNC_ALL(c)                        \
    do {                                   \
        int _rc = sync_all(c);             \
        if (_rc != VO_OK) return _rc;      \
    } while (0)

int read_state(vo_ctx* c, VoState* h)
{
    SYNC_ALL(c);
    HIPCHK(hipMemcpy(h, c->d.st, sizeof(VoState), hipMemcpyDeviceToHost));
    return VO_OK;
}

int read_work0(vo_ctx* c, VoWork* w)
{
    SYNC_ALL(c);
    HIPCHK(hipMemcpy(w, c->d.work, sizeof(VoWork), hipMemcpyDeviceToHost));
    // a bounded in-kernel wait that timed out (k_ransac_fused, k_select_fused) counts in ctr[VO_CTR_ERR]
    uint32_t nerr = 0;
    HIPCHK(hipMemcpy(&nerr, c->d.ctr + VO_CTR_ERR, sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (nerr) {
        fprintf(stderr, "[vo_mi355x] device error counter is %u (a consistency check or bounded wait failed)\n", nerr);
        return VO_ERR_INTERNAL;
    }
    return VO_OK;
}

int write_work0(vo_ctx* c, const VoWork* w)
{
    SYNC_ALL(c);
    HIPCHK(hipMemcpy(c->d.work, w, sizeof(VoWork), hipMemcpyHostToDevice));
    return VO_OK;
}

// work[0] of a stage call: status OK, counters clear
void stage_work(VoWork* w, int ring)
{
    std::memset(w, 0, sizeof(*w));
    w->status = VO_STATUS_OK;
    w->frame = -1;
    w->bestk = -1;
    w->prev = ring + 1;          // the two stage slots after the ring and the carry slot
    w->cur = ring + 2;
}

// the stage RANSAC calls' points: f64 as given, their f32 copy in the count's word layout, and the
// coordinate bounds of the f32 Sampson certificate (rounded up; +inf disables it for the call)
int upload_stage_pts(vo_ctx* c, const VoDev& d, const double* pts, int m, VoWork* w)
{
    HIPCHK(hipMemcpy(d.pts, pts, sizeof(double) * 4 * (size_t)m, hipMemcpyHostToDevice));
    std::vector<float> p32(VO_PTS32_PER(c->cfg.max_kpts), 0.0f);
    double mx[4] = {0.0, 0.0, 0.0, 0.0};
    for (int i = 0; i < m; ++i)
        for (int k = 0; k < 4; ++k) {
            const double v = pts[4 * (size_t)i + k];
            p32[vo_pts32_index(i, k)] = (float)v;
            mx[k] = std::isfinite(v) ? std::max(mx[k], std::fabs(v)) : HUGE_VAL;
        }
    for (int k = 0; k < 4; ++k) {
        float f = (float)mx[k];
        if ((double)f < mx[k]) f = std::nextafter(f, HUGE_VALF);
        w->cmax[k] = f;
    }
    HIPCHK(hipMemcpy(d.pts32, p32.data(), sizeof(float) * p32.size(), hipMemcpyHostToDevice));
    return VO_OK;
}

// host frame (any stride) -> frame_in on stream `st`, via the pinned staging buffer
double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// zero_copy: only stage the frame in the pinned buffer; the caller's stencil reads it there over PCIe
int upload_frame(vo_ctx* c, const uint8_t* gray, size_t stride, hipStream_t st, bool zero_copy = false)
{
    const int W = c->cfg.width, H = c->cfg.height;
    if (stride == 0) stride = (size_t)W;
    const double t0 = c->pf_profile ? now_us() : 0.0;
    SYNC_ALL(c);                          // staging buffer / frame_in may still be in use
    const double t1 = c->pf_profile ? now_us() : 0.0;
    if (stride == (size_t)W) {
        std::memcpy(c->stage_host, gray, (size_t)W * H);
    } else {
        for (int y = 0; y < H; ++y) std::memcpy(c->stage_host + (size_t)y * W, gray + (size_t)y * stride, W);
    }
    // a copy kernel on the frame's own queue reads the pinned staging buffer (a copy-engine transfer
    // measured 15 us plus a ~14 us engine -> compute-queue hand-off before the next kernel)
    if (c->pf_profile) {
        const double t2 = now_us();
        c->pf_t[0] += t1 - t0;
        c->pf_t[1] += t2 - t1;
    }
    if (zero_copy) return VO_OK;
    vo::launch_h2d(c->d.frame_in, c->stage_host, (size_t)W * H, st);
    HIPCHK(hipGetLastError());
    return VO_OK;
}

// stage extract (vo_extract / vo_response): frame_in -> slot VO_STAGE_SLOT, scratch 0
void enqueue_stage_extract(vo_ctx* c)
{
    VoDev d = c->d;
    d.single = 1;                       // one frame: latency-shaped launches
    vo::launch_stencil(d, d.frame_in, 0, 1, 0, c->s);
    vo::launch_select(d, 0, 1, d.ring + 1, c->s);
    vo::launch_describe(d, 0, 1, d.ring + 1, 0u, c->s);
}

// Timing: every timed launch is bracketed by two events on the stream it runs on (all
// kernels, or only kernel `only`); vo_last_kernel_times averages end - start.
struct EvRec {
    std::vector<hipEvent_t>* pool;
    size_t used;
    int only;   // -1: all kernels
    std::vector<int>* launches;
    std::vector<std::pair<int, size_t>> spans;   // (kernel, index of its start event)
    int err = VO_OK;                             // first failed event create / record
};
// An event pair costs ~6 us of queue time per bracketed launch (rocprofv3 kernel trace), so
// the bench's live single-kernel timing samples one launch in VO_TIMING_STRIDE.
#define VO_TIMING_STRIDE 4

size_t ev_mark(EvRec* ev, hipStream_t st)
{
    if (ev->used >= ev->pool->size()) {
        hipEvent_t e = nullptr;
        // device-scope release: a system-scope fence (the default) writes back and invalidates
        // the L2s at every record, which is most of an event's queue cost here
        if (hip_ok(hipEventCreateWithFlags(&e, hipEventReleaseToDevice)) != VO_OK) {
            ev->err = VO_ERR_HIP;
            return SIZE_MAX;
        }
        ev->pool->push_back(e);
    }
    if (hip_ok(hipEventRecord((*ev->pool)[ev->used], st)) != VO_OK) {
        ev->err = VO_ERR_HIP;
        return SIZE_MAX;
    }
    return ev->used++;
}

// event k of the per-batch pool (created on demand)
int batch_event(vo_ctx* c, int pool, size_t k, hipEvent_t* e)
{
    std::vector<hipEvent_t>& v = c->ev_batch[pool];
    while (v.size() <= k) {
        hipEvent_t x = nullptr;
        HIPCHK(hipEventCreateWithFlags(&x, hipEventDisableTiming | hipEventReleaseToDevice));
        v.push_back(x);
    }
    *e = v[k];
    return VO_OK;
}

constexpr int kContSpan = 1000;    // EvRec span tag of a continuation launch (timed, cont)
// cont: the rest of the previous launch of kernel k (a pass's later RANSAC chunks on another
// queue): its time adds to that launch's, which stays one launch in the counts
template <typename F>
void timed(vo_ctx* c, EvRec* ev, int k, hipStream_t st, F&& launch, bool cont = false)
{
    const int nth = cont ? c->klaunch[k] - 1 : c->klaunch[k]++;
    const bool on = ev && ev->err == VO_OK && (ev->only < 0 || (ev->only == k && nth % VO_TIMING_STRIDE == 0));
    size_t b = on ? ev_mark(ev, st) : 0;
    launch();
    if (on && b != SIZE_MAX && ev_mark(ev, st) != SIZE_MAX) ev->spans.emplace_back(cont ? k + kContSpan : k, b);
}

// extract of nb frames f0.. (device images img0 + z * frame_bytes) on stream q; publish:
// the pose queue may wait for frames < f0 + nb
// eq: extract queue index (its scratch copy and counters)
// ev_stencil (optional): recorded on q once the stencil (the only reader of the images) is enqueued
// q2 (optional): select and describe on a second queue after the stencil (event e_s)
// scr: the scratch copy (default eq, the queue's); st_nb: frames of the stencil launch -- nb, 0 (the
// previous batch's paired launch covered this one) or 2 nb (this batch and the next, scratch copies
// scr and scr + 1, which are contiguous)
int enqueue_extract(vo_ctx* c, const uint8_t* img0, size_t frame_bytes, int f0, int nb, bool publish,
                    hipStream_t q, EvRec* ev, int eq, hipEvent_t ev_stencil = nullptr, bool single = false)
{
    VoDev d = c->d;
    d.single = single ? 1 : 0;          // the single-frame call: latency-shaped extract launches
    const size_t B = (size_t)c->Bx;     // the scratch copies' capacity
    const int scr = eq;                 // scratch copy
    const int st_nb = nb;
    d.eq = eq;
    d.diag_f0 = f0;
    d.blurred += d.bplane * B * scr;
    d.cand += (size_t)d.cand_cap * B * scr;
    d.tilerows += (size_t)d.ntiles * 16 * B * scr;
    d.ckeys += (size_t)d.cand_cap * B * scr;
    d.selbits += ((size_t)d.cand_cap / 64 + 1) * B * scr;
    d.selctl += B * scr;
    d.hist += (size_t)VO_HIST_BINS * B * scr;
    if (d.tile_ck) d.tile_ck += (size_t)d.ntiles * B * scr;
    if (st_nb > 0) timed(c, ev, 0, q, [&] { vo::launch_stencil(d, img0, frame_bytes, st_nb, 0, q); });
    if (ev_stencil) HIPCHK(hipEventRecord(ev_stencil, q));
    timed(c, ev, 1, q, [&] { vo::launch_select(d, f0, nb, -1, q); });
    timed(c, ev, 2, q, [&] { vo::launch_describe(d, f0, nb, -1, publish ? (unsigned)(f0 + nb) : 0u, q); });
    return VO_OK;
}

// Host-frame streaming (vo_process_frames_host): batch j of a chunk is copied from host memory
// into device ring slot j % VO_HRING on the copy queue `sc` while earlier batches are extracted
// and posed.  The copy of batch j waits for the stencil of batch j - VO_HRING (the last reader
// of that slot); the stencil of batch j waits for its copy.  Pinned sources are DMA'd directly;
// pageable ones go through the pinned staging ring (the host waits for the copy that last
// used a staging slot before refilling it).
struct HostSrc {
    const uint8_t* frames;    // frame f of the chunk at frames + f * frame_bytes (dense W x H rows)
    size_t frame_bytes;
    bool pinned;              // DMA from the source; else staged through c->hstage
};

int enqueue_h2d(vo_ctx* c, const HostSrc& hs, int f0, int nb, int j, uint8_t** dimg)
{
    const size_t np = (size_t)c->cfg.width * c->cfg.height, slot = (size_t)(j % VO_HRING);
    uint8_t* dst = c->dring + slot * (size_t)c->B * np;
    hipEvent_t e_cp, e_st;
    int rc = batch_event(c, VO_EV_COPY, (size_t)j, &e_cp);
    if (rc) return rc;
    if (j >= VO_HRING) {
        rc = batch_event(c, VO_EV_STENCIL, (size_t)(j - VO_HRING), &e_st);
        if (rc) return rc;
        HIPCHK(hipStreamWaitEvent(c->sc, e_st, 0));
    }
    const uint8_t* src = hs.frames + (size_t)f0 * hs.frame_bytes;
    if (!hs.pinned) {
        // refill staging slot `slot` once its previous copy (batch j - VO_HRING) has run
        if (j >= VO_HRING) {
            hipEvent_t e_prev;
            rc = batch_event(c, VO_EV_COPY, (size_t)(j - VO_HRING), &e_prev);
            if (rc) return rc;
            HIPCHK(hipEventSynchronize(e_prev));
        }
        uint8_t* stg = c->hstage + slot * (size_t)c->B * np;
        for (int z = 0; z < nb; ++z) std::memcpy(stg + (size_t)z * np, src + (size_t)z * hs.frame_bytes, np);
        HIPCHK(hipMemcpyAsync(dst, stg, np * nb, hipMemcpyHostToDevice, c->sc));
    } else if (hs.frame_bytes == np) {
        HIPCHK(hipMemcpyAsync(dst, src, np * nb, hipMemcpyHostToDevice, c->sc));
    } else {
        HIPCHK(hipMemcpy2DAsync(dst, np, src, hs.frame_bytes, np, nb, hipMemcpyHostToDevice, c->sc));
    }
    HIPCHK(hipEventRecord(e_cp, c->sc));
    *dimg = dst;
    return VO_OK;
}

// the window buffers of pass p: set p & 1 (a pipelined pass's match and RANSAC write one set while
// the previous pass's refit, triangulation and finalize read the other)
// The reference's sampler (ransac.cpp:137,142): rng = std::mt19937(seed32) once, then per hypothesis
// k the elements std::sample(data.begin(), data.end(), std::back_inserter(sample), sampleSize, rng)
// picks, as indices into data (selection sampling keeps data order).  The population is an index
// vector with random-access iterators like the reference's vector<pair<Point, Point>>, and the size
// argument an int like its `int sampleSize = 8`, so libstdc++ takes the same code path and draws the
// same numbers (tests/test_reference_sampler.py compiles the reference's own expression against it).
void mt_samples(uint32_t seed32, int m, int nhyp, int32_t* out)
{
    std::mt19937 rng(seed32);
    std::vector<int32_t> idx((size_t)m);
    std::iota(idx.begin(), idx.end(), 0);
    const int sampleSize = 8;
    std::vector<int32_t> smp;
    smp.reserve(8);
    for (int k = 0; k < nhyp; ++k) {
        smp.clear();
        std::sample(idx.begin(), idx.end(), std::back_inserter(smp), sampleSize, rng);
        for (int i = 0; i < 8; ++i) out[8 * (size_t)k + i] = i < (int)smp.size() ? smp[(size_t)i] : 0;
    }
}

// VO_RNG_MT19937: the hypotheses' samples of records [0, nrec) of a pose window, once k_match has
// written the records (status, M, frame seed) -- a host round trip on the pose queue
int upload_mt_samples(vo_ctx* c, const VoDev& d, int nrec, hipStream_t s)
{
    HIPCHK(hipStreamSynchronize(s));
    std::vector<VoWork> w((size_t)nrec);
    HIPCHK(hipMemcpy(w.data(), d.work, sizeof(VoWork) * (size_t)nrec, hipMemcpyDeviceToHost));
    std::vector<int32_t> tab((size_t)d.max_hyp * 8);
    for (int r = 0; r < nrec; ++r) {
        if (w[(size_t)r].status != VO_STATUS_OK || w[(size_t)r].M < 8) continue;
        mt_samples((uint32_t)w[(size_t)r].frame_seed, w[(size_t)r].M, d.max_hyp, tab.data());
        HIPCHK(hipMemcpy(d.samples + (size_t)r * d.max_hyp * 8, tab.data(), tab.size() * sizeof(int32_t),
                         hipMemcpyHostToDevice));
    }
    return VO_OK;
}

VoDev pass_dev(const vo_ctx* c, int p)
{
    VoDev d = c->d;
    if (p & 1) {
        const size_t* o = c->set_off;
        d.match_j += o[0]; d.match_pairs += o[1]; d.pts += o[2]; d.hypF += o[3]; d.counts += o[4];
        d.inl += o[5]; d.inlmask += o[6]; d.model_p += o[7]; d.work += o[8]; d.pts32 += o[9];
    }
    return d;
}

// one pose pass over the window of the frames enqueued so far (up to WB frames; k_match decides
// it on the device, vo_kernels.hip pass_window).  gmax: frames < gmax are extracted once the pass
// runs (its wait covers them).  pipelined: match and RANSAC on the pose queue, refit,
// triangulation and finalize on the fit queue, so the next pass's match overlaps them; the pass
// first waits for pass p - 2's finalize (its buffer set and its state snapshot).  Otherwise every
// kernel on the pose queue and the window comes from the state (every earlier pass finalized).
// first: the chunk's first pass (every earlier pass finalized: its window comes from the state,
// d.nospec) -- pipelined or not, its own window needs no speculation
void enqueue_pass(vo_ctx* c, VoFrameOut* out, int out_base, EvRec* ev, int gmax, bool pipelined, bool single = false,
                  bool first = false)
{
    hipStream_t s = c->s;
    const int p = c->npass++;
    VoDev d = pass_dev(c, p);
    d.gmax = gmax;
    if (single) {
        // one frame per call: its window holds at most two records (a repair window's dual ones)
        d.single = 1;
        d.gridw = std::min(2, d.WB);
    }
    d.pass = p;
    d.nospec = pipelined && !first ? 0 : 1;
    hipStream_t sf = pipelined ? c->sf : s;
    if (pipelined) (void)hipStreamWaitEvent(s, c->ev_fn[(p + vo_ctx::kPassEv - 2) % vo_ctx::kPassEv], 0);
    timed(c, ev, 3, s, [&] { vo::launch_match(d, 0, s); });
    if (d.rng_mode == VO_RNG_MT19937) {
        const int rc = upload_mt_samples(c, d, d.gridw, s);
        if (rc && ev && !ev->err) ev->err = rc;
        if (rc) c->mt_err = rc;
    }
    // pipelined: the later hypothesis chunks run on the fit queue, after the first chunk's replay,
    // so the next pass's match and first chunk overlap them (the pass's buffer set is its own; the
    // reference-sampler mode's sample table is not, so it keeps every chunk on the pose queue)
    static const bool split_env = !(getenv("VO_RANSAC_SPLIT") && atoi(getenv("VO_RANSAC_SPLIT")) == 0);
    const bool split = pipelined && split_env && d.rng_mode != VO_RNG_MT19937;
    timed(c, ev, 4, s, [&] { vo::launch_ransac(d, 0, s, split ? 1 : 0); });
    // c->rq: the later chunks on the trajectory queue instead (the trajectory chain moves to the fit
    // queue), so the next pass's later chunks overlap this pass's refit, triangulation and finalize
    const bool rq = split && c->rq;
    if (pipelined) {
        (void)hipEventRecord(c->ev_rs[p % vo_ctx::kPassEv], s);
        (void)hipStreamWaitEvent(rq ? c->st : sf, c->ev_rs[p % vo_ctx::kPassEv], 0);
    }
    if (rq) {
        timed(c, ev, 4, c->st, [&] { vo::launch_ransac(d, 0, c->st, 2); }, true);
        (void)hipEventRecord(c->ev_r2[p % vo_ctx::kPassEv], c->st);
        (void)hipStreamWaitEvent(sf, c->ev_r2[p % vo_ctx::kPassEv], 0);
    } else if (split) {
        timed(c, ev, 4, sf, [&] { vo::launch_ransac(d, 0, sf, 2); }, true);
    }
    timed(c, ev, 5, sf, [&] { vo::launch_refit(d, 1, 0, sf); });
    if (single) {
        // one frame: triangulation, finalize and the trajectory chain in one launch (its last
        // workgroup), on the pose queue
        timed(c, ev, 6, sf, [&] { vo::launch_triangulate(d, 0, sf, out, out_base, 2); });
        return;
    }
    timed(c, ev, 6, sf, [&] { vo::launch_triangulate(d, 0, sf); });
    timed(c, ev, 7, sf, [&] { vo::launch_finalize(d, out, out_base, sf); });
    // the T_curr chain and the pose rows on the trajectory queue (serial mode and the single-frame
    // call: the pose queue, no cross-queue event)
    hipStream_t q = c->serial || single ? s : (c->rq ? sf : c->st);
    hipEvent_t ef = pipelined ? c->ev_fn[p % vo_ctx::kPassEv] : c->ev_fin;
    if (q != sf || pipelined) {
        (void)hipEventRecord(ef, sf);
        if (q != sf) (void)hipStreamWaitEvent(q, ef, 0);
    }
    timed(c, ev, 8, q, [&] { vo::launch_traj(d, out, out_base, q); });
}

// Batch sizes of a chunk: B frames per extract batch and per pass window (the last one
// shorter).  Pass k's window starts at or before batch k's first frame, so its frames are
// extracted once batch k is.  (Smaller first batches to start the pose queue earlier were
// measured slower: more passes, each with a fixed latency.)
// Host streaming (first_default > 0): the first batch is short, so its H2D copy (the pipeline
// fill: 64 KITTI frames are 30 MB, ~0.5 ms at PCIe's ~56 GB/s) does not hold back the first extract
// (tools/host_stream_diag.py: first batch 8/16/32 measured +5 % over 64).
// cap > B (device frames): a remainder of at most B / 2 frames after a full batch joins that batch
// (up to cap frames) -- a short last batch costs nearly a full batch's extract launches (the stencil,
// the banded select and describe run latency-bound on few frames) and a pose pass of its own
// (VO_TAIL=0: the short batch).  Host streaming keeps B: its device ring slots hold B frames.
std::vector<int> batch_schedule(int nf, int B, int first_default = 0, int cap = 0)
{
    static const bool env_tail = !(getenv("VO_TAIL") && atoi(getenv("VO_TAIL")) == 0);
    // experiment knob: VO_FIRST = size of the first batch (pipeline fill), default B
    static const int env_first = getenv("VO_FIRST") ? atoi(getenv("VO_FIRST")) : -1;
    // experiment knob: VO_LAST = size of the batches the chunk's last B frames are split into (the
    // drain: the last pass covers only the last small batch)
    static const int env_last = getenv("VO_LAST") ? atoi(getenv("VO_LAST")) : 0;
    const int first = env_first >= 0 ? env_first : first_default;
    std::vector<int> v;
    for (int done = 0; done < nf;) {
        int want = (done == 0 && first > 0 && first < B) ? first : B;
        if (env_last > 0 && env_last < B && nf - done <= B) want = env_last;
        else if (env_tail && want == B && nf - done > B && nf - done <= cap && nf - done - B <= B / 2) want = nf - done;
        v.push_back(std::min(want, nf - done));
        done += v.back();
    }
    return v;
}

// frames [c->fidx, c->fidx + nf) (nf <= VO_CHUNK): set the end, enqueue the extract
// batches (img != null: device images; null: one missing image) and one pass per window,
// then repeat passes until every frame is committed (a pass commits at least its first frame)
// hs (optional): host frames streamed through the device ring (img0 unused)
int run_chunk(vo_ctx* c, const uint8_t* img0, size_t frame_bytes, int nf, VoFrameOut* out, int out_base, EvRec* ev,
              bool host_frame, const HostSrc* hs = nullptr)
{
    const int base = c->fidx, end = base + nf, B = c->B;
    hipStream_t s = c->s;
    c->others_busy = true;
    const bool multi = hs || !(c->serial || host_frame || !img0);   // extract on its own queues
    if (multi && c->reset_pending) {
        for (hipStream_t q : c->se)
            if (q) HIPCHK(hipStreamWaitEvent(q, c->ev_reset, 0));
        c->reset_pending = false;
    }
    const std::vector<int> sched = batch_schedule(nf, B, hs ? VO_HOST_FIRST_BATCH : 0, hs ? 0 : c->Bx);
    // extract batch j on its queue (+ its event in event-wait mode)
    std::vector<int> f0s(sched.size() + 1, 0);
    for (size_t j = 0; j < sched.size(); ++j) f0s[j + 1] = f0s[j] + sched[j];

    auto extract = [&](int j) -> int {
        const int f0 = f0s[j], cnt = sched[j];
        // describe publishes the extracted-frame count only for the polling wait kernel
        const bool publish = multi && !c->event_wait;
        hipStream_t q = multi ? c->se[0] : s;
        if (hs) {
            uint8_t* dimg = nullptr;
            hipEvent_t e_cp, e_st;
            int rc = enqueue_h2d(c, *hs, f0, cnt, j, &dimg);
            if (rc == VO_OK) rc = batch_event(c, VO_EV_COPY, (size_t)j, &e_cp);
            if (rc == VO_OK) rc = batch_event(c, VO_EV_STENCIL, (size_t)j, &e_st);
            if (rc) return rc;
            HIPCHK(hipStreamWaitEvent(q, e_cp, 0));
            rc = enqueue_extract(c, dimg, (size_t)c->cfg.width * c->cfg.height, base + f0, cnt, publish, q, ev, 0,
                                 e_st);
            if (rc) return rc;
        } else {
            int rc = enqueue_extract(c, img0 + (size_t)f0 * frame_bytes, frame_bytes, base + f0, cnt, publish, q, ev,
                                     0, nullptr, host_frame);
            if (rc) return rc;
        }
        if (multi && c->event_wait) {
            // the event the pass of this batch waits on.  (The record costs the extract queue ~8 us
            // between a describe and the next stencil, kernel trace r6e; a pose pass per two batches,
            // recording every second event, measured 227-228k vs 298-300k KITTI frames/s: the pose
            // queue then runs in 128-frame bursts, r6f)
            hipEvent_t e;
            int rc = batch_event(c, VO_EV_WAIT, (size_t)j, &e);
            if (rc) return rc;
            HIPCHK(hipEventRecord(e, q));
        }
        return VO_OK;
    };
    // pass k waits for batch k (the extract queue runs batches in order)
    bool first_pass = true;                    // the chunk's first pass (its window from the state)
    auto pass = [&](int k) -> int {
        if (multi) {
            if (!c->event_wait) {
                // one wave on the pose queue polls the frame count describe's last workgroup publishes
                // (bounded: a timeout counts in the error counter, VO_ERR_INTERNAL)
                vo::launch_wait_ext(c->d, (unsigned)(base + f0s[k + 1]), s);
            } else {
                hipEvent_t e;
                int rc = batch_event(c, VO_EV_WAIT, (size_t)k, &e);
                if (rc) return rc;
                HIPCHK(hipStreamWaitEvent(s, e, 0));
            }
        }
        // the chunk's first pass sees every earlier pass finalized (the last call synchronised):
        // its window comes from the state.  Its refit, triangulation and finalize go to the fit
        // queue like every later pass's (the next pass speculates on its window as on any
        // pipelined one's), so pass 1's match need not wait for them (VO_PIPE_FIRST=0: the whole
        // first pass on the pose queue)
        static const bool pipe_first = !(getenv("VO_PIPE_FIRST") && atoi(getenv("VO_PIPE_FIRST")) == 0);
        enqueue_pass(c, out, out_base, ev, base + f0s[k + 1], multi && c->pipeline && (!first_pass || pipe_first),
                     host_frame, first_pass);
        first_pass = false;
        return VO_OK;
    };
    if (!img0 && !hs) {
        vo::launch_ext_missing(c->d, base % c->d.ring, s);
        c->fidx = end;
        int rc = pass(0);
        if (rc) return rc;
    } else {
        // enqueue order: the extract queue one batch ahead of the pose queue, so pass k is
        // queued as soon as batch k is (all extracts first would hold the first pass back by
        // the host time of every extract launch of the chunk)
        int rc = extract(0);
        if (rc) return rc;
        if (c->host_profile) c->hp_t[1] = now_us();
        c->fidx = end;
        for (size_t k = 0; k < sched.size(); ++k) {
            if (k + 1 < sched.size() && (rc = extract((int)k + 1)) != VO_OK) return rc;
            if ((rc = pass((int)k)) != VO_OK) return rc;
        }
        // slack passes: the frames left behind by speculation misses, without a host round trip
        // (a pass with nothing left to commit returns at once); long chunks only
        if (sched.size() >= 4)
            for (int k = 0; k < c->slack; ++k) enqueue_pass(c, out, out_base, ev, end, multi && c->pipeline);
    }
    if (c->host_profile) c->hp_t[2] = now_us();
    // every pass commits at least its first frame, so nf re-pass rounds bound the loop
    for (int round = 0, prev_lo = base;; ++round) {
        HIPCHK(hipGetLastError());
        // the chunk's output rows (complete once the trajectory queue's last k_traj ran, which
        // waited for the last k_finalize) and the commit point
        hipStream_t tq = c->serial || host_frame ? s : (c->rq ? c->sf : c->st);
        // (c->rq: a non-pipelined pass runs its trajectory chain on the pose queue, which the fit
        // queue does not otherwise follow — the re-pass rounds, a missing frame's pass)
        if (c->rq && tq != s) {
            HIPCHK(hipEventRecord(c->ev_fin, s));
            HIPCHK(hipStreamWaitEvent(tq, c->ev_fin, 0));
        }
        if (out != c->out_host_dev)                       // (the per-frame call's kernels wrote out_host itself)
            HIPCHK(hipMemcpyAsync(c->out_host + (base - out_base), out + (base - out_base), sizeof(VoFrameOut) * nf,
                                  hipMemcpyDeviceToHost, tq));
        // the commit point after the last finalize (the fit queue's, which the trajectory queue waited
        // for).  A single frame's pass (window of one, no speculation) commits it: its row is read
        // alone and checked to be that frame's
        if (!host_frame && !(c->d.lo_host_dev && out == c->out_host_dev))
            HIPCHK(hipMemcpyAsync(c->lo_host, &c->d.st->lo, sizeof(int32_t), hipMemcpyDeviceToHost, tq));
        if (c->pf_profile && host_frame) c->pf_enq_end = now_us();
        HIPCHK(hipStreamSynchronize(s));
        if (c->pf_profile && host_frame) c->pf_wait_end = now_us();
        if (c->sf && !host_frame) HIPCHK(hipStreamSynchronize(c->sf));
        if (tq != s) HIPCHK(hipStreamSynchronize(tq));
        if (c->rq && c->st && !host_frame) HIPCHK(hipStreamSynchronize(c->st));
        if (host_frame && nf == 1 && c->out_host[base - out_base].frame != base) {
            fprintf(stderr, "[vo_mi355x] single-frame pass did not commit frame %d\n", base);
            return VO_ERR_STATE;
        }
        const int lo = host_frame && nf == 1 ? end : *c->lo_host;
        if (lo >= end) {
            // every queue is idle: each extract batch's event was waited on by a pass, and the pose, fit
            // and trajectory queues were synchronised above
            c->others_busy = false;
            break;
        }
        if (lo < base || lo > end || round > nf || (round > 0 && lo <= prev_lo)) {
            fprintf(stderr, "[vo_mi355x] pose passes made no progress (committed %d of [%d, %d), round %d)\n", lo,
                    base, end, round);
            return VO_ERR_STATE;
        }
        prev_lo = lo;
        // frames after skipped ones: their windows restart at lo (extracts are complete)
        // (the host synchronised: every pass is finalized, so these run from the state, in order)
        for (int k = 0; k < (end - lo + B - 1) / B; ++k) enqueue_pass(c, out, out_base, ev, end, false, host_frame);
    }
    if (ev && ev->err) return ev->err;
    if (c->mt_err) { const int e = c->mt_err; c->mt_err = 0; return e; }
    // a frame the select's consistency check failed (VO_STATUS_INCONSISTENT): a library defect, loud
    for (int f = base; f < end; ++f)
        if (c->out_host[f - out_base].status == VO_STATUS_INCONSISTENT || c->out_host[f - out_base].err) {
            // err bit 0: the frame's select failed its consistency check; bit 1: the context's device
            // error counter was set when the frame was committed (a bounded in-kernel wait timed out)
            fprintf(stderr, "[vo_mi355x] frame %d: device consistency check failed (err %d)\n", f,
                    c->out_host[f - out_base].err);
            return VO_ERR_INTERNAL;
        }
    return VO_OK;
}

// the context's device consistency failures (ctr[VO_CTR_ERR]) once its queues are idle
int dev_errors(vo_ctx* c, uint32_t* n)
{
    SYNC_ALL(c);
    HIPCHK(hipMemcpy(n, c->d.ctr + VO_CTR_ERR, sizeof(uint32_t), hipMemcpyDeviceToHost));
    return VO_OK;
}

int ensure_out(vo_ctx* c, int n)
{
    if (n <= c->out_cap) return VO_OK;
    if (c->out_dev) (void)hipFree(c->out_dev);
    if (c->out_host) (void)hipHostFree(c->out_host);
    c->out_dev = nullptr; c->out_host = nullptr; c->out_host_dev = nullptr; c->out_cap = 0;
    HIPCHK(hipMalloc((void**)&c->out_dev, sizeof(VoFrameOut) * (size_t)n));
    HIPCHK(hipHostMalloc((void**)&c->out_host, sizeof(VoFrameOut) * (size_t)n, hipHostMallocDefault));
    if (hipHostGetDevicePointer((void**)&c->out_host_dev, c->out_host, 0) != hipSuccess) {
        (void)hipGetLastError();
        c->out_host_dev = nullptr;
    }
    c->out_cap = n;
    return VO_OK;
}

int finish_timing(vo_ctx* c, EvRec* ev)
{
    const int nk = vo::kernel_count();
    c->ktime_ms.assign(nk, 0.f);
    c->kcont_ms.assign(nk, 0.f);
    c->kcount.assign(nk, 0);
    if (!ev) return VO_OK;
    SYNC_ALL(c);
    if (ev->err) return ev->err;
    for (const auto& sp : ev->spans) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, c->ev_pool[sp.second], c->ev_pool[sp.second + 1]);
        const bool cont = sp.first >= kContSpan;
        c->ktime_ms[cont ? sp.first - kContSpan : sp.first] += ms;
        if (cont) c->kcont_ms[sp.first - kContSpan] += ms;
        if (!cont) c->kcount[sp.first] += 1;
    }
    return VO_OK;
}

}  // namespace

extern "C" {

int vo_abi_version(void) { return VO_ABI_VERSION; }

const char* vo_strerror(int code)
{
    switch (code) {
    case VO_OK: return "ok";
    case VO_ERR_ARG: return "invalid argument";
    case VO_ERR_HIP: return "HIP runtime error";
    case VO_ERR_NO_DEVICE: return "no HIP device";
    case VO_ERR_CAPACITY: return "capacity exceeded";
    case VO_ERR_STATE: return "invalid state";
    case VO_ERR_IO: return "image could not be read";
    case VO_ERR_INTERNAL: return "device consistency check failed (library defect)";
    case VO_ERR_DEGENERATE_E: return "Degenerate essential matrix";
    default: return "unknown error";
    }
}

void vo_config_default(vo_config* c, int width, int height)
{
    std::memset(c, 0, sizeof(*c));
    c->width = width; c->height = height;
    c->max_kpts = 2000; c->nms_k = 3; c->resp_thr = 20000.0f;
    c->border_row = 35; c->border_col = 37;
    c->ratio = 0.75f; c->match_bits = 32;
    c->ransac_p = 0.99; c->sampson_thr = 1.0; c->ransac_chunk_threads = 8;
    c->seed = 0xACE0ULL;
    const double K[9] = {7.188560000000e+02, 0, 6.071928000000e+02, 0, 7.188560000000e+02, 1.852157000000e+02, 0, 0, 1.0};
    std::memcpy(c->K, K, sizeof(K));
    c->device = 0;
}

void vo_unpack_descriptor(const uint64_t words[8], uint8_t bytes[512])
{
    for (int t = 0; t < 512; ++t) bytes[t] = (uint8_t)((words[t >> 6] >> (t & 63)) & 1u);
}

int vo_create(const vo_config* cfg, vo_ctx** out)
{
    if (!cfg || !out) return VO_ERR_ARG;
    *out = nullptr;
    const vo_config& k = *cfg;
    if (k.width < 8 || k.height < 8 || k.width > 65535 || k.height > 65535) return VO_ERR_ARG;
    if (k.max_kpts < 1 || k.max_kpts > 4096) return VO_ERR_ARG;
    if (k.nms_k != 3) return VO_ERR_ARG;                     // the VO path uses k = 3
    if (!(k.resp_thr >= 0.0f)) return VO_ERR_ARG;
    if (k.match_bits != 32 && k.match_bits != 512) return VO_ERR_ARG;
    if (!(k.ransac_p > 0.0 && k.ransac_p < 1.0) || k.ransac_chunk_threads < 1) return VO_ERR_ARG;
    if (k.frame_batch < 0 || k.frame_batch > VO_MAX_BATCH) return VO_ERR_ARG;
    if (k.rng_mode != VO_RNG_SPLITMIX && k.rng_mode != VO_RNG_MT19937) return VO_ERR_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return VO_ERR_NO_DEVICE;
    if (k.device < 0 || k.device >= ndev) return VO_ERR_NO_DEVICE;
    if (hip_ok(hipSetDevice(k.device)) != VO_OK) return VO_ERR_HIP;

    vo_ctx* c = new (std::nothrow) vo_ctx();
    if (!c) return VO_ERR_CAPACITY;
    c->cfg = k;
    VoDev& d = c->d;
    std::memset(&d, 0, sizeof(d));
    const int W = k.width, H = k.height, N = k.max_kpts;
    const int B = k.frame_batch ? k.frame_batch : VO_DEFAULT_BATCH;
    c->B = B;
    // extract buffers hold up to Bx frames: a chunk whose remainder after a full batch is at most B / 2
    // frames extracts it with that batch (batch_schedule) instead of as a short batch of its own
    const int Bx = std::min(VO_MAX_BATCH, B + B / 2);
    c->Bx = Bx;
    d.B = Bx;
    d.WB = std::min(VO_MAX_WIN, 2 * B);
    if (getenv("VO_WIN")) d.WB = std::max(1, std::min(VO_MAX_WIN, atoi(getenv("VO_WIN"))));
    d.gridw = d.WB;
    d.single = 0;
    d.gmax = INT_MAX;
    d.W = W; d.H = H; d.N = N;
    d.ring = VO_RING_DEFAULT;
    if (getenv("VO_RING_SLOTS")) d.ring = std::max(2 * VO_MAX_BATCH, std::min(1 << 16, atoi(getenv("VO_RING_SLOTS"))));
    d.nms_k = k.nms_k; d.brow = k.border_row; d.bcol = k.border_col;
    d.resp_thr = k.resp_thr * (float)VO_RESP_SCALE;   // the stencil's responses carry VO_RESP_SCALE
    std::memcpy(&d.thr_bits, &d.resp_thr, 4);
    d.ratio = k.ratio; d.match_bits = k.match_bits;
    d.ransac_p = k.ransac_p; d.sampson_thr = k.sampson_thr; d.T = k.ransac_chunk_threads;
    d.seed = k.seed;
    d.rng_mode = k.rng_mode;                // validated with the other arguments above
    std::memcpy(d.K, k.K, sizeof(d.K));
    {
        double outlierRatio = 0.5;
        d.maxit_initial = to_int_x86(std::log(1.0 - k.ransac_p) / std::log(1.0 - std::pow(1.0 - outlierRatio, 8.0)));
    }
    d.max_hyp = std::max(VO_MAX_HYP, std::min(d.maxit_initial, 1 << 20));
    // stencil tiles of VO_TILE_W x VO_TILE_H, at most VO_TILE_CAP strict maxima each
    const int ntiles = ((W + VO_TILE_W - 1) / VO_TILE_W) * ((H + VO_TILE_H - 1) / VO_TILE_H);
    if (ntiles > 3072) { delete c; return VO_ERR_ARG; }      // SEL_MAX_TILES (select kernel LDS)
    d.ntiles = ntiles;
    d.cand_cap = (uint32_t)ntiles * VO_TILE_CAP;
    int rc = VO_OK;
    auto bail = [&](int r) { vo_destroy(c); return r; };
    c->serial = getenv("VO_SERIAL") && atoi(getenv("VO_SERIAL")) != 0;
    // the pose queue waits for extract batches on events by default (barrier packets the queue
    // processes itself); VO_EVENT_WAIT=0: a one-wave kernel on the pose queue polls the counter
    // describe publishes, so the extract queue records no event (k_wait_ext)
    c->event_wait = !(getenv("VO_EVENT_WAIT") && atoi(getenv("VO_EVENT_WAIT")) == 0);
    d.xcd_map = getenv("VO_XCD") ? atoi(getenv("VO_XCD")) : 1;
    c->pf_profile = getenv("VO_PF_PROFILE") && atoi(getenv("VO_PF_PROFILE")) != 0;
    c->host_profile = getenv("VO_HOST_PROFILE") && atoi(getenv("VO_HOST_PROFILE")) != 0;
    c->pipeline = !c->serial && !(getenv("VO_PIPELINE") && atoi(getenv("VO_PIPELINE")) == 0);
    c->slack = getenv("VO_SLACK") ? std::max(0, std::min(64, atoi(getenv("VO_SLACK")))) : VO_SLACK_DEFAULT;
    d.fault_inject = getenv("VO_FAULT_INJECT") && atoi(getenv("VO_FAULT_INJECT")) != 0;   // tests only
    d.spin_limit = getenv("VO_SPIN_LIMIT") ? (unsigned)atoi(getenv("VO_SPIN_LIMIT")) : (1u << 22);   // tests only
    // the per-frame call's select in one launch (VO_SEL_FUSED=0: two launches).  With acquire polls it
    // was slower (21.2 us against 9.0 + 9.2 us, gpurun_out r5e: each poll invalidated the XCD's L2);
    // with relaxed polls the call is 1.5-1.9 us faster per frame (two alternating pairs, r5i)
    d.sel_fused = !(getenv("VO_SEL_FUSED") && atoi(getenv("VO_SEL_FUSED")) == 0);
    d.ransac_fused = !(getenv("VO_RANSAC_FUSED") && atoi(getenv("VO_RANSAC_FUSED")) == 0);
    // a pipelined pass's later RANSAC chunks on the trajectory queue and the trajectory chain on the
    // fit queue (VO_RANSAC_Q=0: the chunks on the fit queue, the chain on its own queue): 0.12
    // m/frame 168.0-168.6k -> 177.6-186.1k, KITTI within noise (three alternating pairs, r5z)
    c->rq = !(getenv("VO_RANSAC_Q") && atoi(getenv("VO_RANSAC_Q")) == 0);
    // repair windows hold two work records per frame (k_finalize): at most WB / 2 frames
    d.repair_win = std::max(1, std::min(d.WB / 2, getenv("VO_REPAIR_WIN") ? atoi(getenv("VO_REPAIR_WIN")) : VO_REPAIR_WIN_DEFAULT));
    // four queues: pose (c->s), trajectory (c->st), fit (c->sf), extract (c->se[0]) -- a process has four
    // hardware queues (GPU_MAX_HW_QUEUES); a fifth stream would share one and serialise behind its kernels
    auto make_stream = [&](hipStream_t* q) { return hipStreamCreateWithFlags(q, hipStreamNonBlocking); };
    if (hip_ok(make_stream(&c->s)) != VO_OK) return bail(VO_ERR_HIP);
    if (hip_ok(make_stream(&c->st)) != VO_OK) return bail(VO_ERR_HIP);
    if (hip_ok(hipEventCreateWithFlags(&c->ev_fin, hipEventDisableTiming | hipEventReleaseToDevice)) != VO_OK)
        return bail(VO_ERR_HIP);
    if (hip_ok(make_stream(&c->sf)) != VO_OK) return bail(VO_ERR_HIP);
    for (int i = 0; i < vo_ctx::kPassEv; ++i)
        if (hip_ok(hipEventCreateWithFlags(&c->ev_rs[i], hipEventDisableTiming | hipEventReleaseToDevice)) != VO_OK ||
            hip_ok(hipEventCreateWithFlags(&c->ev_fn[i], hipEventDisableTiming | hipEventReleaseToDevice)) != VO_OK ||
            hip_ok(hipEventCreateWithFlags(&c->ev_r2[i], hipEventDisableTiming | hipEventReleaseToDevice)) != VO_OK)
            return bail(VO_ERR_HIP);
    if (hip_ok(make_stream(&c->se[0])) != VO_OK) return bail(VO_ERR_HIP);
    if (hip_ok(hipEventCreateWithFlags(&c->ev_reset, hipEventDisableTiming)) != VO_OK) return bail(VO_ERR_HIP);
    d.sel_lds = vo::select_lds_bytes(W, H, nullptr);
    if (d.sel_lds < 0) return bail(VO_ERR_HIP);
    // select: banded (VO_SEL_BANDS workgroups per frame) from VO_SEL_BANDED_TILES stencil tiles up
    // (1920x1080: select 3.45 -> 1.93 us/frame, 70k -> 78k frames/s), one 1024-thread workgroup per
    // frame below (KITTI's 552 tiles: 0.45 vs 0.48 us/frame, 281-285k vs 276-277k frames/s);
    // VO_SEL1=1 / 0 forces the single-workgroup / banded form.  A band too large for LDS: single.
    d.sel_emit_lds = vo::select_emit_lds_bytes(W, H);
    d.sel1 = getenv("VO_SEL1") ? atoi(getenv("VO_SEL1")) != 0 : ntiles < VO_SEL_BANDED_TILES;
    if (d.sel_emit_lds < 0) d.sel1 = 1;
    // the fused select with its band's keys staged in LDS (VO_SEL_EARLY=0: the emit after the wait)
    if (d.sel_fused && !(getenv("VO_SEL_EARLY") && atoi(getenv("VO_SEL_EARLY")) == 0) && d.sel_emit_lds >= 0 &&
        vo::select_fused_lds_bytes(W, H) > 0)
        d.sel_fused = 2;
    const size_t np = (size_t)W * H;
    rc |= dalloc_rec(c, "frame_in", &d.frame_in, np);
    d.bstride = vo_blur_stride(W);
    d.bplane = (size_t)d.bstride * vo_blur_rows(H);
    rc |= dalloc_rec(c, "blurred", &d.blurred, d.bplane * Bx * VO_EXT_QUEUES);
    rc |= dalloc_rec(c, "response", &d.response, np);
    rc |= dalloc_rec(c, "cand", &d.cand, (size_t)d.cand_cap * Bx * VO_EXT_QUEUES);
    rc |= dalloc_rec(c, "tilerows", &d.tilerows, (size_t)ntiles * 16 * Bx * VO_EXT_QUEUES);
    rc |= dalloc_rec(c, "ckeys", &d.ckeys, (size_t)d.cand_cap * Bx * VO_EXT_QUEUES);
    rc |= dalloc_rec(c, "selbits", &d.selbits, ((size_t)d.cand_cap / 64 + 1) * Bx * VO_EXT_QUEUES);
    rc |= dalloc_rec(c, "hist", &d.hist, (size_t)VO_HIST_BINS * Bx * VO_EXT_QUEUES);
    rc |= dalloc_rec(c, "selctl", &d.selctl, (size_t)Bx * VO_EXT_QUEUES);
    rc |= dalloc_rec(c, "kps", &d.kps, (size_t)N * VO_SLOTS);
    rc |= dalloc_rec(c, "desc", &d.desc, (size_t)N * 8 * VO_SLOTS);
    rc |= dalloc_rec(c, "pre", &d.pre, (size_t)N * VO_SLOTS);
    const int WB = d.WB;                                       // pose window buffers: two sets (pass p uses set p & 1)
    d.mask_words = (N + 63) / 64;
    const size_t per[10] = {(size_t)N * WB, (size_t)N * WB, (size_t)N * 4 * WB, (size_t)d.max_hyp * 9 * WB,
                            (size_t)d.max_hyp * WB, (size_t)N * WB, (size_t)d.max_hyp * d.mask_words * WB,
                            (size_t)N * 4 * WB, (size_t)WB, VO_PTS32_PER(N) * WB};
    std::memcpy(c->set_off, per, sizeof(per));
    rc |= dalloc_rec(c, "match_j", &d.match_j, 2 * per[0]);
    rc |= dalloc_rec(c, "match_pairs", &d.match_pairs, 2 * per[1]);
    rc |= dalloc_rec(c, "pts", &d.pts, 2 * per[2]);
    rc |= dalloc_rec(c, "pts32", &d.pts32, 2 * per[9]);
    rc |= dalloc_rec(c, "hypF", &d.hypF, 2 * per[3]);
    rc |= dalloc_rec(c, "counts", &d.counts, 2 * per[4]);
    rc |= dalloc_rec(c, "inl", &d.inl, 2 * per[5]);
    rc |= dalloc_rec(c, "inlmask", &d.inlmask, 2 * per[6]);
    rc |= dalloc_rec(c, "model_p", &d.model_p, 2 * per[7]);
    rc |= dalloc_rec(c, "work", &d.work, 2 * per[8]);
    if (d.rng_mode == VO_RNG_MT19937) rc |= dalloc_rec(c, "samples", &d.samples, (size_t)d.max_hyp * 8 * WB);
    rc |= dalloc_rec(c, "plan", &d.plan, VO_PASS_RING);
    rc |= dalloc_rec(c, "snap", &d.snap, VO_PASS_RING);
    rc |= dalloc_rec(c, "st", &d.st, 1);
    rc |= dalloc_rec(c, "ext_n", &d.ext_n, VO_SLOTS);
    rc |= dalloc_rec(c, "ext_st", &d.ext_st, VO_SLOTS);
    rc |= dalloc_rec(c, "seq_starts", &d.seq_starts, VO_MAX_SEQ_STARTS);
    rc |= dalloc_rec(c, "ctr", &d.ctr, VO_CTR_WORDS);
    rc |= dalloc_rec(c, "trec", &d.trec, VO_SLOTS);
    rc |= dalloc_rec(c, "plog", &d.plog, VO_PLOG);
#if defined(VO_STAMPS) || (defined(MM_VERIFY) && MM_VERIFY) || ST_DIAG
    rc |= dalloc_rec(c, "dbg", &d.dbg, (size_t)d.max_hyp * 16);   // stamps / diagnostic counters (words 6000..6003)
#endif
#if ST_DIAG
    rc |= dalloc_rec(c, "tile_ck", &d.tile_ck, (size_t)ntiles * Bx * VO_EXT_QUEUES);
    rc |= dalloc_rec(c, "diag_tile", &d.diag_tile, (size_t)ntiles * VO_DIAG_FRAMES);
    rc |= dalloc_rec(c, "diag_src", &d.diag_src, (size_t)ntiles * VO_DIAG_FRAMES);
    rc |= dalloc_rec(c, "diag_resp", &d.diag_resp, (size_t)ntiles * VO_DIAG_FRAMES);
    rc |= dalloc_rec(c, "diag_keys", &d.diag_keys, (size_t)VO_DIAG_KEYS * VO_DIAG_FRAMES);
#endif
    if (rc != VO_OK) return bail(VO_ERR_HIP);
    const auto tabp = maxit_table(N, k.ransac_p);
    const std::vector<uint16_t>& tab = *tabp;
    if (dalloc(&c->tab_dev, tab.size()) != VO_OK) return bail(VO_ERR_HIP);
    if (hip_ok(hipMemcpy(c->tab_dev, tab.data(), tab.size() * sizeof(uint16_t), hipMemcpyHostToDevice)) != VO_OK)
        return bail(VO_ERR_HIP);
    d.maxit_tab = c->tab_dev;
    if (hip_ok(hipHostMalloc((void**)&c->stage_host, np, hipHostMallocDefault)) != VO_OK) return bail(VO_ERR_HIP);
    if (hip_ok(hipHostMalloc((void**)&c->lo_host, sizeof(int32_t), hipHostMallocDefault)) != VO_OK)
        return bail(VO_ERR_HIP);
    // batched calls: the pose rows and the commit point straight into pinned host memory (VO_OUT_ZC=0:
    // device rows and two D2H copies after the last pass, ~25 us at the end of every call, traces tr012c, trkitti)
    d.lo_host_dev = nullptr;
    c->out_zc = !(getenv("VO_OUT_ZC") && atoi(getenv("VO_OUT_ZC")) == 0);
    if (c->out_zc && hipHostGetDevicePointer((void**)&d.lo_host_dev, c->lo_host, 0) != hipSuccess) {
        (void)hipGetLastError();
        d.lo_host_dev = nullptr;
    }
    // deterministic contents before first use
    (void)hipMemset(d.kps, 0, sizeof(int2) * N * VO_SLOTS);
    (void)hipMemset(d.desc, 0, sizeof(uint64_t) * 8 * N * VO_SLOTS);
    (void)hipMemset(d.pre, 0, sizeof(uint32_t) * N * VO_SLOTS);
    (void)hipMemset(d.selctl, 0, sizeof(VoSelCtl) * Bx * VO_EXT_QUEUES);   // arrival / boundary counters
    if (d.dbg) (void)hipMemset(d.dbg, 0, sizeof(unsigned long long) * (size_t)d.max_hyp * 16);
    d.n_seq_starts = 0;
    d.origin = 0;
    if (ensure_out(c, 16) != VO_OK) return bail(VO_ERR_HIP);
    c->klaunch.assign(vo::kernel_count(), 0);
    if (vo_reset(c) != VO_OK) return bail(VO_ERR_HIP);
    if (hip_ok(hipDeviceSynchronize()) != VO_OK) return bail(VO_ERR_HIP);
    *out = c;
    return VO_OK;
}

void vo_destroy(vo_ctx* c)
{
    if (c && c->pf_profile && c->pf_n)
        fprintf(stderr, "[vo_mi355x] vo_process_frame host phases over %ld calls (us/call): sync %.1f copy %.1f "
                        "enqueue %.1f wait %.1f total %.1f\n", c->pf_n, c->pf_t[0] / c->pf_n, c->pf_t[1] / c->pf_n,
                c->pf_t[2] / c->pf_n, c->pf_t[3] / c->pf_n, c->pf_t[4] / c->pf_n);
    if (!c) return;
    (void)hipSetDevice(c->cfg.device);
    for (hipStream_t q : c->se)
        if (q) (void)hipStreamSynchronize(q);
    if (c->s) (void)hipStreamSynchronize(c->s);
    if (c->sf) (void)hipStreamSynchronize(c->sf);
    if (c->st) (void)hipStreamSynchronize(c->st);
    VoDev& d = c->d;
    void* ptrs[] = {d.frame_in, d.blurred, d.response, d.cand, d.tilerows, d.ckeys, d.selbits, d.hist, d.selctl, d.ext_n, d.ext_st, (void*)d.seq_starts,
                    d.kps, d.desc, d.pre, d.match_j, d.match_pairs, d.pts, d.hypF, d.counts, d.inl, d.inlmask,
                    d.model_p, d.work, d.st, (void*)d.gt, c->tab_dev, c->out_dev, d.ctr, d.trec, d.plog, d.dbg,
                    d.plan, d.snap, d.tile_ck, d.diag_tile, d.diag_src, d.diag_resp, d.diag_keys, d.samples};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (c->out_host) (void)hipHostFree(c->out_host);
    if (c->stage_host) (void)hipHostFree(c->stage_host);
    if (c->lo_host) (void)hipHostFree(c->lo_host);
    for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
    for (auto& v : c->ev_batch)
        for (hipEvent_t e : v) (void)hipEventDestroy(e);
    if (c->dring) (void)hipFree(c->dring);
    if (c->hstage) (void)hipHostFree(c->hstage);
    if (c->sc) (void)hipStreamDestroy(c->sc);
    if (c->ev_reset) (void)hipEventDestroy(c->ev_reset);
    for (int i = 0; i < 2; ++i) {
        if (c->ev_meta[i]) (void)hipEventSynchronize(c->ev_meta[i]);
        if (c->ev_meta[i]) (void)hipEventDestroy(c->ev_meta[i]);
        if (c->meta_host[i]) (void)hipHostFree(c->meta_host[i]);
    }
    for (hipEvent_t e : c->ev_meta_q)
        if (e) (void)hipEventDestroy(e);
    for (auto& kv : c->tab_by_p) (void)hipFree(kv.second);
    for (hipStream_t q : c->se)
        if (q && q != c->st) (void)hipStreamDestroy(q);
    if (c->s) (void)hipStreamDestroy(c->s);
    if (c->st) (void)hipStreamDestroy(c->st);
    if (c->ev_fin) (void)hipEventDestroy(c->ev_fin);
    if (c->sf) (void)hipStreamDestroy(c->sf);
    for (int i = 0; i < vo_ctx::kPassEv; ++i) {
        if (c->ev_rs[i]) (void)hipEventDestroy(c->ev_rs[i]);
        if (c->ev_fn[i]) (void)hipEventDestroy(c->ev_fn[i]);
        if (c->ev_r2[i]) (void)hipEventDestroy(c->ev_r2[i]);
    }
    delete c;
}

// Asynchronous: one kernel on the pose queue (every API call ends synchronised, so nothing
// is in flight); the extract queue's next batch waits for it through ev_reset.
int vo_reset(vo_ctx* c)
{
    if (!c) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    VoDev d = c->d;
    d.pass = c->npass;                 // the pass rings start over at the next pass
    vo::launch_reset(d, c->s);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(c->ev_reset, c->s));
    c->reset_pending = true;
    c->fidx = 0;
    return VO_OK;
}

// Host metadata (which = 0: GT rows, 1: sequence starts) to device memory without a host-device
// sync: copied into a pinned staging buffer (the caller's array may go away on return) and from
// there on the pose queue, after every other queue's earlier work.  Every kernel that reads it --
// k_match's sequence bases (pose queue), the trajectory chain's GT scale (behind the pose queue
// through the pass events) -- is enqueued later, so it sees the new values; extract kernels read
// neither.  The staging buffer is rewritten only after its previous upload has run.
int upload_meta(vo_ctx* c, int which, void* dst, const void* src, size_t bytes)
{
    if (!bytes) return VO_OK;
    if (c->ev_meta[which]) HIPCHK(hipEventSynchronize(c->ev_meta[which]));
    else HIPCHK(hipEventCreateWithFlags(&c->ev_meta[which], hipEventDisableTiming));
    if (c->meta_cap[which] < bytes) {
        if (c->meta_host[which]) (void)hipHostFree(c->meta_host[which]);
        c->meta_host[which] = nullptr;
        c->meta_cap[which] = 0;
        HIPCHK(hipHostMalloc(&c->meta_host[which], bytes, hipHostMallocDefault));
        c->meta_cap[which] = bytes;
    }
    std::memcpy(c->meta_host[which], src, bytes);
    hipStream_t others[VO_EXT_QUEUES + 2];
    int no = 0;
    for (hipStream_t q : c->se) others[no++] = q;
    others[no++] = c->sf;
    others[no++] = c->st;
    for (int i = 0; i < no && c->others_busy; ++i) {
        if (!others[i]) continue;
        if (!c->ev_meta_q[i]) HIPCHK(hipEventCreateWithFlags(&c->ev_meta_q[i], hipEventDisableTiming));
        HIPCHK(hipEventRecord(c->ev_meta_q[i], others[i]));
        HIPCHK(hipStreamWaitEvent(c->s, c->ev_meta_q[i], 0));
    }
    HIPCHK(hipMemcpyAsync(dst, c->meta_host[which], bytes, hipMemcpyHostToDevice, c->s));
    HIPCHK(hipEventRecord(c->ev_meta[which], c->s));
    return VO_OK;
}

int vo_set_sequence_starts(vo_ctx* c, const int32_t* starts, int n)
{
    if (!c || n < 0 || n > VO_MAX_SEQ_STARTS || (n > 0 && !starts)) return VO_ERR_ARG;
    for (int i = 0; i < n; ++i)
        if (starts[i] < 1 || (i > 0 && starts[i] <= starts[i - 1])) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    const int rc = upload_meta(c, 1, (void*)c->d.seq_starts, starts, sizeof(int32_t) * (size_t)n);
    if (rc) return rc;
    c->d.n_seq_starts = n;
    return VO_OK;
}

int vo_set_frame_origin(vo_ctx* c, int origin)
{
    if (!c || origin < 0) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    SYNC_ALL(c);
    c->d.origin = origin;
    return VO_OK;
}

int vo_ring_slots(vo_ctx* c)
{
    if (!c) return VO_ERR_ARG;
    return c->d.ring;
}

int vo_trajectory_state(vo_ctx* c, double Tcurr[16])
{
    if (!c || !Tcurr) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    SYNC_ALL(c);
    HIPCHK(hipMemcpy(Tcurr, c->d.st->Tcurr, sizeof(double) * 16, hipMemcpyDeviceToHost));
    return VO_OK;
}

// the chain of committed frames [f0, f0 + n) from T_in, in windows of VO_MAX_WIN frames on the
// trajectory queue (k_traj_range); their trajectory records must still be in the ring
int vo_rechain(vo_ctx* c, const double T_in[16], int f0, int n, double* poses_out)
{
    if (!c || !T_in || f0 < 0 || n < 0) return VO_ERR_ARG;
    if (f0 + n > c->fidx || f0 < c->fidx - c->d.ring) return VO_ERR_STATE;
    HIPCHK(hipSetDevice(c->cfg.device));
    SYNC_ALL(c);
    int rc = ensure_out(c, std::max(n, 1));
    if (rc) return rc;
    HIPCHK(hipMemcpy(c->d.st->Tcurr, T_in, sizeof(double) * 16, hipMemcpyHostToDevice));
    for (int lo = f0; lo < f0 + n; lo += VO_MAX_WIN)
        vo::launch_traj_range(c->d, c->out_dev, f0, lo, std::min(VO_MAX_WIN, f0 + n - lo), c->st);
    HIPCHK(hipGetLastError());
    if (n) HIPCHK(hipMemcpyAsync(c->out_host, c->out_dev, sizeof(VoFrameOut) * (size_t)n, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    for (int f = 0; f < n && poses_out; ++f) std::memcpy(poses_out + 12 * (size_t)f, c->out_host[f].pose, sizeof(double) * 12);
    return VO_OK;
}

int vo_set_ground_truth(vo_ctx* c, const double* poses12, int n)
{
    if (!c || n < 0 || (n > 0 && !poses12)) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    if (n > c->gt_cap) {
        SYNC_ALL(c);                                   // the old rows may still be read
        if (c->d.gt) (void)hipFree((void*)c->d.gt);
        double* g = nullptr;
        HIPCHK(hipMalloc((void**)&g, sizeof(double) * 12 * (size_t)n));
        c->d.gt = g;
        c->gt_cap = n;
    }
    const int rc = upload_meta(c, 0, (void*)c->d.gt, poses12, sizeof(double) * 12 * (size_t)n);
    if (rc) return rc;
    c->d.gt_n = n;
    return VO_OK;
}

int vo_extract(vo_ctx* c, const uint8_t* gray, size_t stride, vo_kp* kps, uint64_t* desc, int* n, uint8_t* blurred)
{
    if (!c || !gray || !n) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    int rc = upload_frame(c, gray, stride, c->s);
    if (rc) return rc;
    enqueue_stage_extract(c);      // stage slot ring + 1: the trajectory's slots are untouched
    HIPCHK(hipGetLastError());
    SYNC_ALL(c);
    int32_t nk = 0, status = 0;
    const size_t stg = (size_t)c->d.ring + 1;
    HIPCHK(hipMemcpy(&nk, &c->d.ext_n[stg], sizeof(int32_t), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&status, &c->d.ext_st[stg], sizeof(int32_t), hipMemcpyDeviceToHost));
    if (status == VO_STATUS_INCONSISTENT) return VO_ERR_INTERNAL;
    if (status != VO_STATUS_OK) return VO_ERR_CAPACITY;
    *n = nk;
    const size_t N = (size_t)c->cfg.max_kpts;
    if (kps && nk) HIPCHK(hipMemcpy(kps, c->d.kps + stg * N, sizeof(vo_kp) * nk, hipMemcpyDeviceToHost));
    if (desc && nk)
        HIPCHK(hipMemcpy(desc, c->d.desc + stg * N * 8, sizeof(uint64_t) * 8 * nk, hipMemcpyDeviceToHost));
    if (blurred)
        HIPCHK(hipMemcpy2D(blurred, (size_t)c->cfg.width, c->d.blurred + VO_BLUR_X0, (size_t)c->d.bstride, (size_t)c->cfg.width,
                           (size_t)c->cfg.height, hipMemcpyDeviceToHost));
    return VO_OK;
}

int vo_response(vo_ctx* c, const uint8_t* gray, size_t stride, float* R)
{
    if (!c || !gray || !R) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    int rc = upload_frame(c, gray, stride, c->s);
    if (rc) return rc;
    const size_t np = (size_t)c->cfg.width * c->cfg.height;
    HIPCHK(hipMemsetAsync(c->d.response, 0, np * sizeof(float), c->s));
    vo::launch_stencil(c->d, c->d.frame_in, 0, 1, getenv("VO_DBG") ? atoi(getenv("VO_DBG")) : 1, c->s);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(R, c->d.response, np * sizeof(float), hipMemcpyDeviceToHost, c->s));
    // the stencil histogram is consumed by select; nothing selects here, so clear it
    HIPCHK(hipMemsetAsync(c->d.hist, 0, sizeof(uint32_t) * VO_HIST_BINS, c->s));
    HIPCHK(hipStreamSynchronize(c->s));
    return VO_OK;
}

int vo_match(vo_ctx* c, const uint64_t* d_prev, int n_prev, const uint64_t* d_cur, int n_cur, vo_match_t* out, int* m)
{
    if (!c || !m || n_prev < 0 || n_cur < 0 || n_prev > c->cfg.max_kpts || n_cur > c->cfg.max_kpts) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    *m = 0;
    if (n_prev == 0 || n_cur == 0) return VO_OK;   // feature_matching_parallel.cpp:57
    std::vector<uint32_t> p0(n_prev), p1(n_cur);
    for (int i = 0; i < n_prev; ++i) p0[i] = (uint32_t)d_prev[8 * (size_t)i];
    for (int i = 0; i < n_cur; ++i) p1[i] = (uint32_t)d_cur[8 * (size_t)i];
    SYNC_ALL(c);
    const size_t N = (size_t)c->cfg.max_kpts;
    const int a = c->d.ring + 1, b = c->d.ring + 2;     // stage slots: the trajectory's stay intact
    HIPCHK(hipMemcpy(c->d.desc + a * N * 8, d_prev, sizeof(uint64_t) * 8 * n_prev, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d.desc + b * N * 8, d_cur, sizeof(uint64_t) * 8 * n_cur, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d.pre + a * N, p0.data(), sizeof(uint32_t) * n_prev, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d.pre + b * N, p1.data(), sizeof(uint32_t) * n_cur, hipMemcpyHostToDevice));
    const int nk2[2] = {n_prev, n_cur};
    HIPCHK(hipMemcpy(c->d.ext_n + a, nk2, sizeof(nk2), hipMemcpyHostToDevice));
    VoWork w;
    stage_work(&w, c->d.ring);
    int rc = write_work0(c, &w);
    if (rc) return rc;
    vo::launch_match(c->d, 1, c->s);
    HIPCHK(hipGetLastError());
    rc = read_work0(c, &w);
    if (rc) return rc;
    *m = w.M;
    if (out && w.M) HIPCHK(hipMemcpy(out, c->d.match_pairs, sizeof(vo_match_t) * w.M, hipMemcpyDeviceToHost));
    return VO_OK;
}

int vo_ransac_F(vo_ctx* c, const double* pts, int m, uint64_t seed, double F[9], int* fitted, int32_t* inlier_idx,
                int* n_inl, int* best_k, int* n_evaluated, int32_t* counts)
{
    if (!c || !pts || m < 8 || m > c->cfg.max_kpts) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    SYNC_ALL(c);
    VoWork w;
    stage_work(&w, c->d.ring);
    int rc = upload_stage_pts(c, c->d, pts, m, &w);
    if (rc) return rc;
    w.M = m;
    w.scored = (m / c->cfg.ransac_chunk_threads) * c->cfg.ransac_chunk_threads;
    w.frame_seed = seed;
    rc = write_work0(c, &w);
    if (rc) return rc;
    if (c->d.rng_mode == VO_RNG_MT19937 && (rc = upload_mt_samples(c, c->d, 1, c->s)) != VO_OK) return rc;
    vo::launch_ransac(c->d, 1, c->s);
    vo::launch_refit(c->d, 0, 1, c->s);
    HIPCHK(hipGetLastError());
    rc = read_work0(c, &w);
    if (rc) return rc;
    // the model persists across calls like FundamentalMatrix model (VisualOdometry.cpp:49)
    if (w.fitted) std::memcpy(c->stage_F, w.F, sizeof(c->stage_F));
    if (F) std::memcpy(F, c->stage_F, sizeof(c->stage_F));
    if (fitted) *fitted = w.fitted;
    if (n_inl) *n_inl = w.n_inl;
    if (best_k) *best_k = w.bestk;
    if (n_evaluated) *n_evaluated = w.n_eval;
    if (inlier_idx && w.bestk >= 0 && w.n_inl > 0)
        HIPCHK(hipMemcpy(inlier_idx, c->d.inl, sizeof(int32_t) * w.n_inl, hipMemcpyDeviceToHost));
    if (counts && w.n_eval > 0)
        HIPCHK(hipMemcpy(counts, c->d.counts, sizeof(int32_t) * std::min(w.n_eval, VO_MAX_HYP), hipMemcpyDeviceToHost));
    return VO_OK;
}

int vo_ransac_run(vo_ctx* c, const double* pts, int m, double probability, double sampson_thr, int num_threads,
                  uint64_t seed, double F[9], int* fitted, int32_t* inlier_idx, int* n_inl, int* n_evaluated)
{
    if (!c || !pts || m < 8 || m > c->cfg.max_kpts || num_threads < 1) return VO_ERR_ARG;
    if (!(probability > 0.0 && probability < 1.0) || !(sampson_thr >= 0.0)) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    // ransac.cpp:129-131: the initial bound for this probability; the hypothesis buffers hold max_hyp
    VoDev d = c->d;
    d.maxit_initial = to_int_x86(std::log(1.0 - probability) / std::log(1.0 - std::pow(1.0 - 0.5, 8.0)));
    if (d.maxit_initial > d.max_hyp) return VO_ERR_CAPACITY;
    d.sampson_thr = sampson_thr;
    d.T = num_threads;
    SYNC_ALL(c);
    if (probability != c->cfg.ransac_p) {
        // one device table besides cfg.ransac_p's: the last other probability's (the device is idle here)
        auto it = c->tab_by_p.find(probability);
        if (it == c->tab_by_p.end()) {
            for (auto& kv : c->tab_by_p) (void)hipFree(kv.second);
            c->tab_by_p.clear();
            const auto tab = maxit_table(c->cfg.max_kpts, probability);
            uint16_t* t = nullptr;
            HIPCHK(hipMalloc((void**)&t, tab->size() * sizeof(uint16_t)));
            HIPCHK(hipMemcpy(t, tab->data(), tab->size() * sizeof(uint16_t), hipMemcpyHostToDevice));
            it = c->tab_by_p.emplace(probability, t).first;
        }
        d.maxit_tab = it->second;
    }
    VoWork w;
    stage_work(&w, d.ring);
    int rc = upload_stage_pts(c, d, pts, m, &w);
    if (rc) return rc;
    w.M = m;
    w.scored = (m / num_threads) * num_threads;        // ransac.cpp:152-157 (quirk 7)
    w.frame_seed = seed;
    rc = write_work0(c, &w);
    if (rc) return rc;
    if (d.rng_mode == VO_RNG_MT19937 && (rc = upload_mt_samples(c, d, 1, c->s)) != VO_OK) return rc;
    vo::launch_ransac(d, 1, c->s);
    vo::launch_refit(d, 0, 1, c->s);
    HIPCHK(hipGetLastError());
    rc = read_work0(c, &w);
    if (rc) return rc;
    if (fitted) *fitted = w.fitted;
    if (F && w.fitted) std::memcpy(F, w.F, sizeof(w.F));
    if (n_inl) *n_inl = w.n_inl;
    if (n_evaluated) *n_evaluated = w.n_eval;
    if (inlier_idx && w.bestk >= 0 && w.n_inl > 0)
        HIPCHK(hipMemcpy(inlier_idx, c->d.inl, sizeof(int32_t) * w.n_inl, hipMemcpyDeviceToHost));
    return VO_OK;
}

int vo_fit_F(vo_ctx* c, const double* pts, int n, double F[9])
{
    if (!c || !pts || !F || n < 8 || n > c->cfg.max_kpts) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    SYNC_ALL(c);
    HIPCHK(hipMemcpy(c->d.pts, pts, sizeof(double) * 4 * (size_t)n, hipMemcpyHostToDevice));
    // every point is an inlier of "hypothesis 0" (k_refit compacts the refit set from its mask)
    std::vector<uint64_t> mask((size_t)c->d.mask_words, 0ull);
    for (int i = 0; i < n; ++i) mask[(size_t)i >> 6] |= 1ull << (i & 63);
    HIPCHK(hipMemcpy(c->d.inlmask, mask.data(), sizeof(uint64_t) * mask.size(), hipMemcpyHostToDevice));
    VoWork w;
    stage_work(&w, c->d.ring);
    w.M = n;
    w.scored = n;
    w.bestk = 0;
    w.cold = 1;
    int rc = write_work0(c, &w);
    if (rc) return rc;
    vo::launch_refit(c->d, 0, 1, c->s);
    HIPCHK(hipGetLastError());
    rc = read_work0(c, &w);
    if (rc) return rc;
    if (!w.fitted) return VO_ERR_STATE;
    std::memcpy(F, w.F, sizeof(w.F));
    return VO_OK;
}

int vo_pose(vo_ctx* c, const double F[9], const float* p1, const float* p2, int n, double scale, double R[9],
            double t[3], int32_t* counts4)
{
    if (!c || !F || !p1 || !p2 || n < 8 || n > c->cfg.max_kpts) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    std::vector<float> mp((size_t)n * 4);
    for (int i = 0; i < n; ++i) {
        mp[4 * i] = p1[2 * i]; mp[4 * i + 1] = p1[2 * i + 1];
        mp[4 * i + 2] = p2[2 * i]; mp[4 * i + 3] = p2[2 * i + 1];
    }
    SYNC_ALL(c);
    HIPCHK(hipMemcpy(c->d.model_p, mp.data(), sizeof(float) * mp.size(), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(&c->d.st->scale_override, &scale, sizeof(double), hipMemcpyHostToDevice));
    VoWork w;
    stage_work(&w, c->d.ring);
    w.fitted = 1;
    w.n_fit = n;
    std::memcpy(w.F, F, sizeof(w.F));
    int rc = write_work0(c, &w);
    if (rc) return rc;
    vo::launch_pose_stage(c->d, 0, c->s);
    vo::launch_triangulate(c->d, 1, c->s);
    vo::launch_pose_stage(c->d, 1, c->s);
    HIPCHK(hipGetLastError());
    VoState h;
    rc = read_state(c, &h);
    if (rc) return rc;
    rc = read_work0(c, &w);
    if (rc) return rc;
    int ret = VO_OK;
    if (h.pose_status == VO_STATUS_DEGENERATE) ret = VO_ERR_DEGENERATE_E;
    else if (h.pose_status != VO_STATUS_OK) ret = VO_ERR_STATE;
    if (ret == VO_OK) {
        if (R) std::memcpy(R, h.pose_R, sizeof(h.pose_R));
        if (t) std::memcpy(t, h.pose_t, sizeof(h.pose_t));
    }
    if (counts4) std::memcpy(counts4, w.counts4, sizeof(w.counts4));
    return ret;
}

int vo_process_frame(vo_ctx* c, const uint8_t* gray, size_t stride, double pose_out[12], int* status, int32_t* info)
{
    if (!c) return VO_ERR_ARG;
    const double t0 = c->pf_profile ? now_us() : 0.0;
    HIPCHK(hipSetDevice(c->cfg.device));
    // the stencil reads the frame from the pinned staging buffer itself, over PCIe, instead of an
    // upload kernel copying it to device memory first (1.8-4.7 us less per call in four alternating
    // pairs, gpurun_out pf_a / pf_z); the next call's staging copy waits for this one (upload_frame's
    // sync).  VO_PF_ZEROCOPY=0: the upload kernel
    static const bool zc = !(getenv("VO_PF_ZEROCOPY") && atoi(getenv("VO_PF_ZEROCOPY")) == 0);
    // a caller frame already in pinned host memory (vo_host_alloc / hipHostRegister) with rows
    // packed: the stencil reads it where it lies, no staging copy (VO_PF_PINNED_DIRECT=0: staged)
    static const bool direct_ok = !(getenv("VO_PF_PINNED_DIRECT") && atoi(getenv("VO_PF_PINNED_DIRECT")) == 0);
    const uint8_t* src = nullptr;
    if (gray && zc && direct_ok && (stride == 0 || stride == (size_t)c->cfg.width)) {
        hipPointerAttribute_t a;
        if (hipPointerGetAttributes(&a, gray) == hipSuccess) {
            if (a.type == hipMemoryTypeHost && a.devicePointer) src = static_cast<const uint8_t*>(a.devicePointer);
        } else {
            (void)hipGetLastError();
        }
    }
    const bool gray_staged = gray && !src;
    if (src) {
        SYNC_ALL(c);                  // nothing of an earlier batched call still in flight
    } else if (gray) {
        int rc = upload_frame(c, gray, stride, c->s, zc);
        if (rc) return rc;
        src = zc ? c->stage_host : c->d.frame_in;
    }
    const double t1 = c->pf_profile ? now_us() : 0.0;
    if (c->pf_profile && !gray_staged) c->pf_t[0] += t1 - t0;   // (direct: the pointer query and the sync)
    const int f = c->fidx;
    // one frame: extract on the pose queue, a window of one (no speculation)
    // the frame's output row straight into pinned host memory (VO_PF_OUT_ZC=0: a device row and a copy)
    static const bool out_zc = !(getenv("VO_PF_OUT_ZC") && atoi(getenv("VO_PF_OUT_ZC")) == 0);
    VoFrameOut* out = out_zc && c->out_host_dev ? c->out_host_dev : c->out_dev;
    int rc = run_chunk(c, src, 0, 1, out, f, nullptr, true);
    if (rc) return rc;
    if (c->pf_profile) {
        c->pf_t[2] += c->pf_enq_end - t1;
        c->pf_t[3] += c->pf_wait_end - c->pf_enq_end;
        c->pf_t[4] += now_us() - t0;
        c->pf_n += 1;
    }
    const VoFrameOut& o = c->out_host[0];
    if (pose_out) std::memcpy(pose_out, o.pose, sizeof(o.pose));
    if (status) *status = o.status;
    if (info) {
        info[0] = o.n_kps; info[1] = o.n_matches; info[2] = o.n_inl; info[3] = o.best_k;
        info[4] = o.n_eval; info[5] = o.fitted; info[6] = 0; info[7] = 0;
    }
    return o.status == VO_STATUS_DEGENERATE ? VO_ERR_DEGENERATE_E : VO_OK;
}

}  // extern "C"

namespace {
// the host-side results of the last nframes frames of a batched call
void copy_results(vo_ctx* c, int nframes, double* poses_out, int* status_out, int32_t* info_out)
{
    for (int f = 0; f < nframes; ++f) {
        const VoFrameOut& o = c->out_host[f];
        if (poses_out) std::memcpy(poses_out + 12 * (size_t)f, o.pose, sizeof(o.pose));
        if (status_out) status_out[f] = o.status;
        if (info_out) {
            int32_t* p = info_out + 8 * (size_t)f;
            p[0] = o.n_kps; p[1] = o.n_matches; p[2] = o.n_inl; p[3] = o.best_k;
            p[4] = o.n_eval; p[5] = o.fitted; p[6] = o.frame; p[7] = 0;
        }
    }
}

// frames of one batched call: device frames (dev) or host frames (host, streamed)
int run_frames(vo_ctx* c, const uint8_t* dev, const uint8_t* host, bool pinned, size_t frame_bytes, int nframes,
               double* poses_out, int* status_out, int32_t* info_out)
{
    if (c->host_profile) c->hp_t[0] = now_us();
    int rc = ensure_out(c, std::max(nframes, 1));
    if (rc) return rc;
    c->klaunch.assign(vo::kernel_count(), 0);
    EvRec rec{&c->ev_pool, 0, c->timing >= 100 ? c->timing - 100 : -1, &c->klaunch, {}};
    EvRec* evp = c->timing ? &rec : nullptr;
    const int base = c->fidx;
    const int chunk = c->d.ring - 1;
    const int pass0 = c->npass;
    for (int f0 = 0; f0 < nframes; f0 += chunk) {
        const int nf = std::min(chunk, nframes - f0);
        VoFrameOut* out = c->out_zc && c->out_host_dev && c->d.lo_host_dev ? c->out_host_dev : c->out_dev;
        if (host) {
            const HostSrc hs{host + (size_t)f0 * frame_bytes, frame_bytes, pinned};
            rc = run_chunk(c, nullptr, frame_bytes, nf, out, base, evp, false, &hs);
        } else {
            rc = run_chunk(c, dev + (size_t)f0 * frame_bytes, frame_bytes, nf, out, base, evp, false);
        }
        if (rc) return rc;
    }
    rc = finish_timing(c, evp);
    if (rc) return rc;
    // diagnostic (VO_PLAN_DUMP=1): each pose pass of the call as (first frame, frames committed)
    static const bool plan_dump = getenv("VO_PLAN_DUMP") && atoi(getenv("VO_PLAN_DUMP")) != 0;
    if (plan_dump && c->npass > pass0 && c->npass - pass0 <= VO_PLOG) {
        std::vector<int2> lg(VO_PLOG);
        HIPCHK(hipMemcpy(lg.data(), c->d.plog, sizeof(int2) * VO_PLOG, hipMemcpyDeviceToHost));
        fprintf(stderr, "[vo_mi355x] passes of the call (lo:committed):");
        for (int p = pass0; p < c->npass; ++p) fprintf(stderr, " %d:%d", lg[p % VO_PLOG].x, lg[p % VO_PLOG].y);
        fprintf(stderr, "\n");
    }
    c->last_frames = nframes;
    copy_results(c, nframes, poses_out, status_out, info_out);
    if (c->host_profile)
        fprintf(stderr, "[vo_mi355x] host: first extract enqueued +%.1f us, all passes +%.1f us, done +%.1f us\n",
                c->hp_t[1] - c->hp_t[0], c->hp_t[2] - c->hp_t[0], now_us() - c->hp_t[0]);
    return VO_OK;
}

// host streaming resources, allocated on first use
int ensure_streaming(vo_ctx* c, bool staging)
{
    const size_t ring = (size_t)VO_HRING * c->B * c->cfg.width * c->cfg.height;
    if (!c->sc) HIPCHK(hipStreamCreateWithFlags(&c->sc, hipStreamNonBlocking));
    if (!c->dring) HIPCHK(hipMalloc((void**)&c->dring, ring));
    if (staging && !c->hstage) HIPCHK(hipHostMalloc((void**)&c->hstage, ring, hipHostMallocDefault));
    return VO_OK;
}

bool is_pinned(const void* p)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}
}  // namespace

extern "C" {

int vo_process_frames_device(vo_ctx* c, const uint8_t* d_frames, size_t frame_bytes, int nframes, double* poses_out,
                             int* status_out, int32_t* info_out)
{
    if (!c || !d_frames || nframes < 0) return VO_ERR_ARG;
    if (frame_bytes < (size_t)c->cfg.width * c->cfg.height) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    return run_frames(c, d_frames, nullptr, false, frame_bytes, nframes, poses_out, status_out, info_out);
}

int vo_process_frames_host(vo_ctx* c, const uint8_t* frames, size_t frame_bytes, int nframes, double* poses_out,
                           int* status_out, int32_t* info_out)
{
    if (!c || nframes < 0 || (nframes > 0 && !frames)) return VO_ERR_ARG;
    const size_t np = (size_t)c->cfg.width * c->cfg.height;
    if (frame_bytes < np) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    if (nframes == 0) return VO_OK;
    bool pinned = is_pinned(frames), registered = false;
    // VO_HOST_STAGING=1: never register pageable sources (tests the staging ring)
    const bool staging_only = getenv("VO_HOST_STAGING") && atoi(getenv("VO_HOST_STAGING")) != 0;
    if (!pinned && !staging_only) {
        // pageable: pin the call's frames for DMA (one registration per call), else stage them
        void* p = const_cast<uint8_t*>(frames);
        if (hipHostRegister(p, (size_t)(nframes - 1) * frame_bytes + np, hipHostRegisterDefault) == hipSuccess) {
            pinned = registered = true;
        } else {
            (void)hipGetLastError();
        }
    }
    int rc = ensure_streaming(c, !pinned);
    if (rc == VO_OK) rc = run_frames(c, nullptr, frames, pinned, frame_bytes, nframes, poses_out, status_out, info_out);
    if (registered) {
        if (rc == VO_OK) rc = sync_all(c);
        if (c->sc) (void)hipStreamSynchronize(c->sc);
        if (hipHostUnregister(const_cast<uint8_t*>(frames)) != hipSuccess && rc == VO_OK) rc = VO_ERR_HIP;
    }
    return rc;
}

int vo_extract_frames_device(vo_ctx* c, const uint8_t* d_frames, size_t frame_bytes, int nframes, vo_kp* kps,
                             uint64_t* desc, int32_t* n_kps)
{
    if (!c || !d_frames || nframes < 0) return VO_ERR_ARG;
    if (frame_bytes < (size_t)c->cfg.width * c->cfg.height) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    // the extract batches run on the pose queue, after the reset kernel (the ring is reused)
    int rc = vo_reset(c);
    if (rc) return rc;
    c->reset_pending = false;
    c->klaunch.assign(vo::kernel_count(), 0);
    EvRec rec{&c->ev_pool, 0, c->timing >= 100 ? c->timing - 100 : -1, &c->klaunch, {}};
    EvRec* evp = c->timing ? &rec : nullptr;
    const size_t N = (size_t)c->cfg.max_kpts;
    for (int f0 = 0; f0 < nframes; f0 += c->d.ring) {
        const int nf = std::min(c->d.ring, nframes - f0);
        int off = 0;
        for (int cnt : batch_schedule(nf, c->B, 0, c->Bx)) {
            rc = enqueue_extract(c, d_frames + (size_t)(f0 + off) * frame_bytes, frame_bytes, off, cnt, false, c->s,
                                 evp, 0);
            if (rc) return rc;
            off += cnt;
        }
        HIPCHK(hipGetLastError());
        if (n_kps || kps || desc) {
            HIPCHK(hipStreamSynchronize(c->s));
            std::vector<int32_t> nk(nf), stt(nf);
            HIPCHK(hipMemcpy(nk.data(), c->d.ext_n, sizeof(int32_t) * nf, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(stt.data(), c->d.ext_st, sizeof(int32_t) * nf, hipMemcpyDeviceToHost));
            for (int z = 0; z < nf; ++z) {
                const size_t f = (size_t)(f0 + z);
                if (stt[z] == VO_STATUS_INCONSISTENT) return VO_ERR_INTERNAL;
                if (stt[z] != VO_STATUS_OK) return VO_ERR_CAPACITY;
                if (n_kps) n_kps[f] = nk[z];
                if (kps && nk[z])
                    HIPCHK(hipMemcpyAsync(kps + f * N, c->d.kps + (size_t)z * N, sizeof(vo_kp) * nk[z],
                                          hipMemcpyDeviceToHost, c->s));
                if (desc && nk[z])
                    HIPCHK(hipMemcpyAsync(desc + f * N * 8, c->d.desc + (size_t)z * N * 8, sizeof(uint64_t) * 8 * nk[z],
                                          hipMemcpyDeviceToHost, c->s));
            }
        }
    }
    HIPCHK(hipStreamSynchronize(c->s));
    rc = finish_timing(c, evp);
    if (rc) return rc;
    c->last_frames = nframes;
    uint32_t nerr = 0;               // read before the reset clears the counter
    if ((rc = dev_errors(c, &nerr)) != VO_OK) return rc;
    rc = vo_reset(c);                // the ring no longer holds the trajectory's descriptors
    if (rc) return rc;
    if (nerr) {
        fprintf(stderr, "[vo_mi355x] %u frames failed the select consistency check\n", nerr);
        return VO_ERR_INTERNAL;
    }
    return VO_OK;
}

int vo_reference_samples(uint32_t seed32, int m, int nhyp, int32_t* out)
{
    if (m < 8 || nhyp < 0 || (nhyp > 0 && !out)) return VO_ERR_ARG;
    mt_samples(seed32, m, nhyp, out);
    return VO_OK;
}

int vo_device_error_count(vo_ctx* c, uint32_t* count)
{
    if (!c || !count) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    return dev_errors(c, count);
}

int vo_host_alloc(vo_ctx* c, size_t bytes, void** hptr)
{
    if (!c || !hptr) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    HIPCHK(hipHostMalloc(hptr, std::max<size_t>(bytes, 1), hipHostMallocDefault));
    return VO_OK;
}

int vo_host_free(vo_ctx* c, void* hptr)
{
    if (!c) return VO_ERR_ARG;
    if (hptr) HIPCHK(hipHostFree(hptr));
    return VO_OK;
}

int vo_enable_kernel_timing(vo_ctx* c, int on)
{
    if (!c) return VO_ERR_ARG;
    if (on != 0 && on != 1 && !(on >= 100 && on < 100 + vo::kernel_count())) return VO_ERR_ARG;
    c->timing = on;
    return VO_OK;
}

int vo_last_kernel_times(vo_ctx* c, const char** names, float* ms, int cap)
{
    return vo_last_kernel_stats(c, names, ms, nullptr, cap);
}

int vo_last_kernel_stats(vo_ctx* c, const char** names, float* ms_per_launch, float* frames_per_launch, int cap)
{
    if (!c) return VO_ERR_ARG;
    int nk = std::min<int>((int)c->ktime_ms.size(), cap);
    for (int k = 0; k < nk; ++k) {
        if (names) names[k] = vo::kernel_name(k);
        if (ms_per_launch) ms_per_launch[k] = c->kcount[k] ? c->ktime_ms[k] / (float)c->kcount[k] : -1.f;
        if (frames_per_launch)
            frames_per_launch[k] = c->klaunch[k] ? (float)c->last_frames / (float)c->klaunch[k] : 0.f;
    }
    // one more entry: "ransac_pose", the part of a pass's RANSAC on the pose queue (its first chunk; the
    // later chunks run on the trajectory or fit queue as continuation spans of the same timed launch)
    constexpr int kR = 4;                             // "ransac"
    if (nk == vo::kernel_count() && cap > nk && (int)c->kcont_ms.size() > kR) {
        if (names) names[nk] = "ransac_pose";
        if (ms_per_launch)
            ms_per_launch[nk] = c->kcount[kR] ? (c->ktime_ms[kR] - c->kcont_ms[kR]) / (float)c->kcount[kR] : -1.f;
        if (frames_per_launch)
            frames_per_launch[nk] = c->klaunch[kR] ? (float)c->last_frames / (float)c->klaunch[kR] : 0.f;
        ++nk;
    }
    return nk;
}

// the kernel symbol(s) (base names, comma-separated) that stage k of the batched path launches in
// this context, k as vo_last_kernel_stats numbers the stages: which rows of a rocprofv3 summary of
// the same run belong to the stage (the matcher has four forms, the select two)
const char* vo_kernel_form(vo_ctx* c, int k)
{
    if (!c || k < 0 || k >= vo::kernel_count()) return nullptr;
    return vo::kernel_form(c->d, k);
}

// diagnostics: copy the stamp buffer (VO_STAMPS builds; returns 0 entries otherwise)
int vo_debug_stamps(vo_ctx* c, unsigned long long* out, int n)
{
    if (!c || !c->d.dbg) return 0;
    int m = std::min(n, c->d.max_hyp * 16);
    HIPCHK(hipStreamSynchronize(c->s));
    HIPCHK(hipMemcpy(out, c->d.dbg, sizeof(unsigned long long) * m, hipMemcpyDeviceToHost));
    return m;
}

// diagnostics (tools/det_stress.py): the ring slots of frames [f0, f0 + n) as the last call left
// them -- keypoint counts, keypoints (n x N int2) and 32-test prefixes (n x N u32)
// device buffer i of the context (name, address, bytes), i = 0 .. count - 1; returns the count
// (i out of range: only the count).  Diagnostics: which buffer a device address falls in.
extern "C" int vo_debug_layout(vo_ctx* c, int i, const char** name, uint64_t* ptr, uint64_t* bytes)
{
    if (!c) return VO_ERR_ARG;
    const int n = (int)c->layout.size();
    if (i >= 0 && i < n) {
        if (name) *name = c->layout[i].name;
        if (ptr) *ptr = c->layout[i].ptr;
        if (bytes) *bytes = c->layout[i].bytes;
    }
    return n;
}

// ST_DIAG builds: rows [f0, f0 + n) of diagnostic array `what` (0 diag_tile, 1 diag_src, 2 diag_resp:
// ntiles words per frame; 3 diag_keys: VO_DIAG_KEYS words per frame).  Returns the words per frame.
extern "C" int vo_debug_diag(vo_ctx* c, int what, int f0, int n, unsigned long long* out)
{
    if (!c) return VO_ERR_ARG;
    const VoDev& d = c->d;
    unsigned long long* src[4] = {d.diag_tile, d.diag_src, d.diag_resp, d.diag_keys};
    if (what < 0 || what > 3 || !src[what]) return 0;
    const size_t per = what == 3 ? (size_t)VO_DIAG_KEYS : (size_t)d.ntiles;
    if (f0 < 0 || n < 0 || f0 + n > VO_DIAG_FRAMES) return VO_ERR_ARG;
    SYNC_ALL(c);
    if (out && n) HIPCHK(hipMemcpy(out, src[what] + (size_t)f0 * per, per * n * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    return (int)per;
}

extern "C" int vo_debug_ring(vo_ctx* c, int f0, int n, int32_t* nk, int32_t* kps, uint32_t* pre)
{
    if (!c || f0 < 0 || n <= 0 || n > c->d.ring || !nk || !kps || !pre) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    HIPCHK(hipDeviceSynchronize());
    const size_t N = (size_t)c->cfg.max_kpts;
    for (int i = 0; i < n; ++i) {
        const int slot = (f0 + i) % c->d.ring;
        HIPCHK(hipMemcpy(nk + i, c->d.ext_n + slot, sizeof(int32_t), hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(kps + (size_t)i * N * 2, c->d.kps + (size_t)slot * N, sizeof(int32_t) * 2 * N, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(pre + (size_t)i * N, c->d.pre + (size_t)slot * N, sizeof(uint32_t) * N, hipMemcpyDeviceToHost));
    }
    return VO_OK;
}

int vo_device_alloc(vo_ctx* c, size_t bytes, void** dptr)
{
    if (!c || !dptr) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    HIPCHK(hipMalloc(dptr, std::max<size_t>(bytes, 1)));
    return VO_OK;
}

int vo_device_free(vo_ctx* c, void* dptr)
{
    if (!c) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    HIPCHK(hipStreamSynchronize(c->s));
    if (dptr) HIPCHK(hipFree(dptr));
    return VO_OK;
}

int vo_device_upload(vo_ctx* c, void* dptr, const void* src, size_t bytes)
{
    if (!c || !dptr || !src) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    HIPCHK(hipMemcpy(dptr, src, bytes, hipMemcpyHostToDevice));
    return VO_OK;
}

// test hook: the refit's null-vector solver (k_refit's ls_nullvec9_par) on n 9x9 matrices
int vo_selftest_nullvec9(const double* S, const double* x0, double* f, int32_t* status, int n, int device)
{
    if (n <= 0 || !S || !x0 || !f || !status) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(device));
    double *dS, *dx, *df;
    int* dst;
    HIPCHK(hipMalloc((void**)&dS, sizeof(double) * 81 * n));
    HIPCHK(hipMalloc((void**)&dx, sizeof(double) * 9 * n));
    HIPCHK(hipMalloc((void**)&df, sizeof(double) * 9 * n));
    HIPCHK(hipMalloc((void**)&dst, sizeof(int) * n));
    HIPCHK(hipMemcpy(dS, S, sizeof(double) * 81 * n, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dx, x0, sizeof(double) * 9 * n, hipMemcpyHostToDevice));
    vo::launch_selftest_nullvec9(dS, dx, df, dst, n, nullptr);
    HIPCHK(hipGetLastError());
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(f, df, sizeof(double) * 9 * n, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(status, dst, sizeof(int) * n, hipMemcpyDeviceToHost));
    (void)hipFree(dS); (void)hipFree(dx); (void)hipFree(df); (void)hipFree(dst);
    return VO_OK;
}


// test hook: device arithmetic self-test (sqrtf, f32 '/', f64 sqrt and '/', det-math)
int vo_selftest_arith(const float* fa, const float* fb, float* fo, const double* da, const double* db, double* dout,
                      int n, int device)
{
    if (n <= 0) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(device));
    float *a, *b, *o;
    double *x, *y, *z;
    HIPCHK(hipMalloc((void**)&a, n * 4)); HIPCHK(hipMalloc((void**)&b, n * 4)); HIPCHK(hipMalloc((void**)&o, n * 16));
    HIPCHK(hipMalloc((void**)&x, n * 8)); HIPCHK(hipMalloc((void**)&y, n * 8)); HIPCHK(hipMalloc((void**)&z, n * 32));
    HIPCHK(hipMemcpy(a, fa, n * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(b, fb, n * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(x, da, n * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(y, db, n * 8, hipMemcpyHostToDevice));
    vo::launch_selftest_arith(a, b, o, x, y, z, n, nullptr);
    HIPCHK(hipGetLastError());
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(fo, o, n * 16, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(dout, z, n * 32, hipMemcpyDeviceToHost));
    (void)hipFree(a); (void)hipFree(b); (void)hipFree(o); (void)hipFree(x); (void)hipFree(y); (void)hipFree(z);
    return VO_OK;
}

}  // extern "C"
