// vo_api.cpp -- host side of libvo_mi355x.so: the C ABI of include/vo_mi355x.h.
//
// One vo_ctx = one GPU + two HIP streams + every device buffer of the path allocated
// once (HBM layout: vo_internal.h).  Per frame the host only enqueues kernels; all
// per-frame decisions of the reference's trajectory loop (skip on < 8 matches /
// inliers, descriptor carry-forward, RANSAC model leak, GT scale) are taken on the
// device from VoState, so frames can be enqueued back to back with no host sync.
//
// Frame pipeline: extract(f) (stencil, select, describe) runs on stream `se` and waits
// only for frame f-2's pose chain; the pose chain of frame f (match, RANSAC, refit,
// triangulate + finalize) runs on stream `s` after extract(f).  So extract(f+1)
// overlaps pose(f).  Three keypoint/descriptor slots make that safe: select(f) picks a
// slot that is neither frame f-1's nor its prev (VoExt, k_select).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <climits>
#include <map>
#include <mutex>
#include <new>
#include <utility>
#include <vector>

#include "vo_internal.h"
#include "../../include/vo_mi355x.h"


struct vo_ctx {
    vo_config cfg;
    VoDev d;
    hipStream_t s = nullptr;          // pose chain (and stage APIs)
    hipStream_t se[VO_EXT_QUEUES] = {};   // extract queues of the frame pipeline
    struct Scratch {                  // per extract queue (queue 0 uses VoDev's own buffers)
        uint8_t* blurred = nullptr;
        uint64_t* cand = nullptr;
        uint8_t* tilerows = nullptr;
        uint64_t* ckeys = nullptr;
        uint64_t* selbits = nullptr;
        uint32_t* hist = nullptr;
    } xs[VO_EXT_QUEUES];
    int fidx = 0;                     // frames enqueued since vo_reset
    uint32_t ext_ready = 0;           // extract seq the last enqueued finalize waits for
    bool serial = false;              // VO_SERIAL=1: every kernel on one queue, no cross-queue
                                      // waits (for profilers that serialize dispatches: PMC passes)
    int max_hyp = VO_MAX_HYP;
    int gt_cap = 0;
    VoFrameOut* out_dev = nullptr;
    int out_cap = 0;
    VoFrameOut* out_host = nullptr;   // pinned
    uint8_t* stage_host = nullptr;    // pinned frame staging
    uint16_t* tab_dev = nullptr;
    int timing = 0;                   // 0 off, 1 all kernels, 100+k only kernel k
    std::vector<hipEvent_t> ev_pool;
    std::vector<float> ktime_ms;
    std::vector<int> kcount;
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
std::mutex g_tab_mu;
std::map<std::pair<int, double>, std::vector<uint16_t>> g_tab_cache;

const std::vector<uint16_t>& maxit_table(int N, double prob)
{
    std::lock_guard<std::mutex> lk(g_tab_mu);
    auto key = std::make_pair(N, prob);
    auto it = g_tab_cache.find(key);
    if (it != g_tab_cache.end()) return it->second;
    std::vector<uint16_t> tab((size_t)(N + 1) * (N + 2) / 2, 0xFFFFu);
    const double lp = std::log(1.0 - prob);
    for (int M = 8; M <= N; ++M) {
        uint16_t* row = tab.data() + (size_t)M * (M + 1) / 2;
        for (int best = 1; best <= M; ++best) {
            double outlierRatio = 1.0 - (double)best / (double)M;
            double denom = std::log(1.0 - std::pow(1.0 - outlierRatio, 8.0));
            if (denom == 0.0) { row[best] = 0xFFFFu; continue; }
            int v = to_int_x86(lp / denom);
            v = std::min(std::max(v, 100), 2000);
            row[best] = (uint16_t)v;
        }
    }
    return g_tab_cache.emplace(key, std::move(tab)).first->second;
}

template <typename T>
int dalloc(T** p, size_t n)
{
    return hip_ok(hipMalloc((void**)p, std::max<size_t>(n, 1) * sizeof(T)));
}

int sync_ext(vo_ctx* c)
{
    for (hipStream_t q : c->se)
        if (q) HIPCHK(hipStreamSynchronize(q));
    return VO_OK;
}
#define SYNC_EXT(c)                        \
    do {                                   \
        int _rc = sync_ext(c);             \
        if (_rc != VO_OK) return _rc;      \
    } while (0)

int read_state(vo_ctx* c, VoState* h)
{
    SYNC_EXT(c);
    HIPCHK(hipMemcpyAsync(h, c->d.st, sizeof(VoState), hipMemcpyDeviceToHost, c->s));
    HIPCHK(hipStreamSynchronize(c->s));
    return VO_OK;
}
int write_state(vo_ctx* c, const VoState* h)
{
    HIPCHK(hipMemcpyAsync(c->d.st, h, sizeof(VoState), hipMemcpyHostToDevice, c->s));
    HIPCHK(hipStreamSynchronize(c->s));
    return VO_OK;
}

int read_ext(vo_ctx* c, VoExt* h)
{
    SYNC_EXT(c);
    HIPCHK(hipMemcpyAsync(h, c->d.ext, sizeof(VoExt), hipMemcpyDeviceToHost, c->s));
    HIPCHK(hipStreamSynchronize(c->s));
    return VO_OK;
}

// host frame (any stride) -> frame_in on stream `st`, via the pinned staging buffer
int upload_frame(vo_ctx* c, const uint8_t* gray, size_t stride, hipStream_t st)
{
    const int W = c->cfg.width, H = c->cfg.height;
    if (stride == 0) stride = (size_t)W;
    HIPCHK(hipStreamSynchronize(c->s));   // staging buffer / frame_in may still be in use
    SYNC_EXT(c);
    if (stride == (size_t)W) {
        std::memcpy(c->stage_host, gray, (size_t)W * H);
    } else {
        for (int y = 0; y < H; ++y) std::memcpy(c->stage_host + (size_t)y * W, gray + (size_t)y * stride, W);
    }
    HIPCHK(hipMemcpyAsync(c->d.frame_in, c->stage_host, (size_t)W * H, hipMemcpyHostToDevice, st));
    return VO_OK;
}

// stage extract (vo_extract): slot VO_STAGE_SLOT, on the pose stream
void enqueue_extract(vo_ctx* c, const uint8_t* dframe, int write_response)
{
    vo::launch_stencil(c->d, dframe, write_response, c->s);
    vo::launch_select(c->d, -1, c->s);
    vo::launch_describe(c->d, -1, c->s);
}

// stage calls borrow the ctx; they restore the trajectory state (and the zeroed
// histogram / arrival counters the next frame expects) afterwards
int restore_state(vo_ctx* c, const VoState* saved)
{
    HIPCHK(hipMemsetAsync(c->d.hist, 0, sizeof(uint32_t) * VO_HIST_BINS, c->s));   // queue 0's
    HIPCHK(hipMemsetAsync(c->d.ctr, 0, sizeof(unsigned) * VO_CTR_COUNTERS, c->s));
    return write_state(c, saved);
}

// the full trajectory-loop iteration for one frame (VisualOdometry.cpp:68-189).
// Timing: every timed kernel is bracketed by two events on the stream it runs on (all
// kernels, or only kernel `only`); vo_last_kernel_times averages end - start.
struct EvRec {
    std::vector<hipEvent_t>* pool;
    size_t used;
    int only;   // -1: all kernels
    int frame;  // frame being enqueued; single-kernel mode brackets every VO_TIMING_STRIDE-th frame
    std::vector<std::pair<int, size_t>> spans;   // (kernel, index of its start event)
};
// An event pair costs ~6 us of queue time per bracketed launch (rocprofv3 kernel trace), so
// the bench's live single-kernel timing samples one frame in VO_TIMING_STRIDE.
#define VO_TIMING_STRIDE 8

size_t ev_mark(EvRec* ev, hipStream_t st)
{
    if (ev->used >= ev->pool->size()) {
        hipEvent_t e;
        // device-scope release: a system-scope fence (the default) writes back and invalidates
        // the L2s at every record, which is most of an event's queue cost here
        (void)hipEventCreateWithFlags(&e, hipEventReleaseToDevice);
        ev->pool->push_back(e);
    }
    (void)hipEventRecord((*ev->pool)[ev->used], st);
    return ev->used++;
}

template <typename F>
void timed(EvRec* ev, int k, hipStream_t st, F&& launch)
{
    const bool on = ev && (ev->only < 0 || (ev->only == k && ev->frame % VO_TIMING_STRIDE == 0));
    size_t b = on ? ev_mark(ev, st) : 0;
    launch();
    if (on) {
        ev_mark(ev, st);
        ev->spans.emplace_back(k, b);
    }
}

// more: the caller enqueues frame f+1 right after this one (the batch path)
void enqueue_frame(vo_ctx* c, const uint8_t* dframe, VoFrameOut* out, EvRec* ev, bool more)
{
    const int f = c->fidx++;
    if (ev) ev->frame = f;
    VoDev d = c->d;
    d.out = out;
    // Cross-queue order by frame counters the kernels publish (describe's last workgroup:
    // frame f extracted; finalize: pose chain done).  An event record + wait costs ~11-18 us
    // of queue time per hop on MI355X (tools/evtest.hip); a stream-wait-value packet on a
    // kernel-written counter ~1-6 us (ROCclr runs it as a small wait kernel); a poll inside
    // the consuming kernel ~1 us.
    const uint32_t seq = (uint32_t)f + 1u;
    d.seqno = seq;
    // extract queue q = f % E with its own scratch; frames on different queues overlap
    const int q = f % VO_EXT_QUEUES;
    hipStream_t se = c->serial ? c->s : c->se[q];
    d.eq = q;
    if (q > 0) {
        const vo_ctx::Scratch& x = c->xs[q];
        d.blurred = x.blurred; d.cand = x.cand; d.tilerows = x.tilerows;
        d.ckeys = x.ckeys; d.selbits = x.selbits; d.hist = x.hist;
    }
    // ring slot f % R is read by the pose chains of frames f - R (cur) and f - R + 1 (prev,
    // or the carry copy finalize(f - R + 1) makes): frame f - R + 1's chain must be done
    if (f >= VO_RING_SLOTS - 1 && !c->serial)
        (void)hipStreamWaitValue32(se, c->d.ctr + VO_SYNC_POSE, seq - (uint32_t)(VO_RING_SLOTS - 1),
                                   hipStreamWaitValueGte, 0xFFFFFFFFu);
    if (dframe) {
        timed(ev, 0, se, [&] { vo::launch_stencil(d, dframe, 0, se); });
        timed(ev, 1, se, [&] { vo::launch_select(d, f, se); });
        timed(ev, 2, se, [&] { vo::launch_describe(d, f, se); });
    } else {
        vo::launch_ext_missing(d, f, se);
    }
    // The pose queue needs frame f's extract before k_match.  Inside a batch the previous
    // frame's finalize (one workgroup) waited for it at its end, so k_match starts behind a
    // kernel boundary with the descriptors in place; otherwise a stream-wait-value packet.
    // (A poll inside k_match itself can deadlock: 250 spinning workgroups can hold the CUs
    // the extract's single 1024-thread select workgroup needs.)
    if (c->ext_ready != seq && !c->serial)
        (void)hipStreamWaitValue32(c->s, c->d.ctr + VO_SYNC_EXT + (f & (VO_EXT_RING - 1)), seq, hipStreamWaitValueGte,
                                   0xFFFFFFFFu);
    d.wait_next = more && !c->serial ? seq + 1u : 0u;
    c->ext_ready = d.wait_next;
    if (dframe) {
        timed(ev, 3, c->s, [&] { vo::launch_match(d, c->s); });
        timed(ev, 4, c->s, [&] { vo::launch_ransac(d, c->max_hyp, c->s); });
        timed(ev, 5, c->s, [&] { vo::launch_refit(d, 1, c->s); });
        timed(ev, 6, c->s, [&] { vo::launch_triangulate(d, c->s); });
    } else {
        vo::launch_missing(d, c->s);
    }
}

int ensure_out(vo_ctx* c, int n)
{
    if (n <= c->out_cap) return VO_OK;
    if (c->out_dev) (void)hipFree(c->out_dev);
    if (c->out_host) (void)hipHostFree(c->out_host);
    c->out_dev = nullptr; c->out_host = nullptr; c->out_cap = 0;
    HIPCHK(hipMalloc((void**)&c->out_dev, sizeof(VoFrameOut) * (size_t)n));
    HIPCHK(hipHostMalloc((void**)&c->out_host, sizeof(VoFrameOut) * (size_t)n, hipHostMallocDefault));
    c->out_cap = n;
    return VO_OK;
}

void init_state(vo_ctx* c, VoState* h)
{
    std::memset(h, 0, sizeof(*h));
    h->frame = 0;
    h->status = VO_STATUS_OK;
    h->cur = 0; h->prev = 0;
    h->bestk = -1;
    h->scale_override = std::nan("");
    for (int i = 0; i < 16; ++i) h->Tcurr[i] = (i % 5 == 0) ? 1.0 : 0.0;
    (void)c;
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
    d.W = W; d.H = H; d.N = N;
    d.nms_k = k.nms_k; d.brow = k.border_row; d.bcol = k.border_col;
    d.resp_thr = k.resp_thr;
    std::memcpy(&d.thr_bits, &k.resp_thr, 4);
    d.ratio = k.ratio; d.match_bits = k.match_bits;
    d.ransac_p = k.ransac_p; d.sampson_thr = k.sampson_thr; d.T = k.ransac_chunk_threads;
    d.seed = k.seed;
    std::memcpy(d.K, k.K, sizeof(d.K));
    {
        double outlierRatio = 0.5;
        d.maxit_initial = to_int_x86(std::log(1.0 - k.ransac_p) / std::log(1.0 - std::pow(1.0 - outlierRatio, 8.0)));
    }
    c->max_hyp = std::max(VO_MAX_HYP, std::min(d.maxit_initial, 1 << 20));
    const int ntiles = ((W + 63) / 64) * ((H + 15) / 16);
    if (ntiles > 2048) { delete c; return VO_ERR_ARG; }      // SEL_MAX_TILES (select kernel LDS)
    d.cand_cap = (uint32_t)ntiles * 256u;
    int rc = VO_OK;
    auto bail = [&](int r) { vo_destroy(c); return r; };
    // no stream priorities: k_match waits inside the kernel for the extract queue, and a
    // high-priority queue spinning on low-priority work can starve it (observed: the wait ran
    // into its timeout when 250 match workgroups were pending at high priority)
    c->serial = getenv("VO_SERIAL") && atoi(getenv("VO_SERIAL")) != 0;
    const char* cu_env = getenv("VO_CU_POSE");
    const int cu_pose = cu_env ? atoi(cu_env) : 0;
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, k.device);
    if (cu_pose > 0 && cu_pose < ncu && ncu <= 1024) {
        // experimental: disjoint CU sets for the two queues (CU ids spread evenly)
        std::vector<uint32_t> mp((ncu + 31) / 32, 0u), me((ncu + 31) / 32, 0u);
        for (int i = 0; i < ncu; ++i) {
            const bool pose = (long)(i + 1) * cu_pose / ncu != (long)i * cu_pose / ncu;
            (pose ? mp : me)[i >> 5] |= 1u << (i & 31);
        }
        if (hip_ok(hipExtStreamCreateWithCUMask(&c->s, (uint32_t)mp.size(), mp.data())) != VO_OK) return bail(VO_ERR_HIP);
        for (hipStream_t& q : c->se)
            if (hip_ok(hipExtStreamCreateWithCUMask(&q, (uint32_t)me.size(), me.data())) != VO_OK) return bail(VO_ERR_HIP);
    } else {
        if (hip_ok(hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking)) != VO_OK) return bail(VO_ERR_HIP);
        for (hipStream_t& q : c->se)
            if (hip_ok(hipStreamCreateWithFlags(&q, hipStreamNonBlocking)) != VO_OK) return bail(VO_ERR_HIP);
    }
    d.sel_lds = vo::select_lds_bytes(W, H, nullptr);
    if (d.sel_lds < 0) return bail(VO_ERR_HIP);
    rc |= dalloc(&d.frame_in, (size_t)W * H);
    rc |= dalloc(&d.blurred, (size_t)W * H);
    rc |= dalloc(&d.response, (size_t)W * H);
    rc |= dalloc(&d.cand, d.cand_cap);
    rc |= dalloc(&d.tilerows, (size_t)ntiles * 16);
    rc |= dalloc(&d.ckeys, d.cand_cap);
    rc |= dalloc(&d.selbits, d.cand_cap / 64 + 1);
    rc |= dalloc(&d.hist, VO_HIST_BINS);
    for (int q = 1; q < VO_EXT_QUEUES; ++q) {
        vo_ctx::Scratch& x = c->xs[q];
        rc |= dalloc(&x.blurred, (size_t)W * H);
        rc |= dalloc(&x.cand, d.cand_cap);
        rc |= dalloc(&x.tilerows, (size_t)ntiles * 16);
        rc |= dalloc(&x.ckeys, d.cand_cap);
        rc |= dalloc(&x.selbits, d.cand_cap / 64 + 1);
        rc |= dalloc(&x.hist, VO_HIST_BINS);
    }
    for (int s = 0; s < VO_SLOTS; ++s) {
        rc |= dalloc(&d.kps[s], N);
        rc |= dalloc(&d.desc[s], (size_t)N * 8);
        rc |= dalloc(&d.pre[s], N);
    }
    rc |= dalloc(&d.match_j, N);
    rc |= dalloc(&d.match_pairs, N);
    rc |= dalloc(&d.pts, (size_t)N * 4);
    rc |= dalloc(&d.hypF, (size_t)c->max_hyp * 9);
    rc |= dalloc(&d.counts, c->max_hyp);
    rc |= dalloc(&d.inl, N);
    d.mask_words = (N + 63) / 64;
    rc |= dalloc(&d.inlmask, (size_t)c->max_hyp * d.mask_words);
    rc |= dalloc(&d.model_p, (size_t)N * 4);
    rc |= dalloc(&d.st, 1);
    rc |= dalloc(&d.ext, 1);
    rc |= dalloc(&d.ctr, VO_CTR_WORDS);
#ifdef VO_STAMPS
    rc |= dalloc(&d.dbg, (size_t)c->max_hyp * 16);
#endif
    if (rc != VO_OK) return bail(VO_ERR_HIP);
    const std::vector<uint16_t>& tab = maxit_table(N, k.ransac_p);
    if (dalloc(&c->tab_dev, tab.size()) != VO_OK) return bail(VO_ERR_HIP);
    if (hip_ok(hipMemcpy(c->tab_dev, tab.data(), tab.size() * sizeof(uint16_t), hipMemcpyHostToDevice)) != VO_OK)
        return bail(VO_ERR_HIP);
    d.maxit_tab = c->tab_dev;
    if (hip_ok(hipHostMalloc((void**)&c->stage_host, (size_t)W * H, hipHostMallocDefault)) != VO_OK) return bail(VO_ERR_HIP);
    // zero the descriptor / keypoint slots (deterministic contents before first use)
    for (int s = 0; s < VO_SLOTS; ++s) {
        (void)hipMemset(d.kps[s], 0, sizeof(int2) * N);
        (void)hipMemset(d.desc[s], 0, sizeof(uint64_t) * 8 * N);
        (void)hipMemset(d.pre[s], 0, sizeof(uint32_t) * N);
    }
    if (ensure_out(c, 16) != VO_OK) return bail(VO_ERR_HIP);
    (void)hipMemset(d.ctr, 0, sizeof(unsigned) * VO_CTR_WORDS);
    if (vo_reset(c) != VO_OK) return bail(VO_ERR_HIP);
    if (hip_ok(hipDeviceSynchronize()) != VO_OK) return bail(VO_ERR_HIP);
    *out = c;
    return VO_OK;
}

void vo_destroy(vo_ctx* c)
{
    if (!c) return;
    (void)hipSetDevice(c->cfg.device);
    for (hipStream_t q : c->se)
        if (q) (void)hipStreamSynchronize(q);
    if (c->s) (void)hipStreamSynchronize(c->s);
    VoDev& d = c->d;
    for (int s = 0; s < VO_SLOTS; ++s) {
        void* sp[] = {d.kps[s], d.desc[s], d.pre[s]};
        for (void* p : sp)
            if (p) (void)hipFree(p);
    }
    void* ptrs[] = {d.frame_in, d.blurred, d.response, d.cand, d.tilerows, d.ckeys, d.selbits, d.hist, d.ext,
                    d.match_j, d.match_pairs, d.pts, d.hypF, d.counts, d.inl, d.inlmask, d.model_p,
                    d.st, (void*)d.gt, c->tab_dev, c->out_dev, d.ctr, d.dbg};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    for (const vo_ctx::Scratch& x : c->xs) {
        void* xp[] = {x.blurred, x.cand, x.tilerows, x.ckeys, x.selbits, x.hist};
        for (void* p : xp)
            if (p) (void)hipFree(p);
    }
    if (c->out_host) (void)hipHostFree(c->out_host);
    if (c->stage_host) (void)hipHostFree(c->stage_host);
    for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
    for (hipStream_t q : c->se)
        if (q) (void)hipStreamDestroy(q);
    if (c->s) (void)hipStreamDestroy(c->s);
    delete c;
}

int vo_reset(vo_ctx* c)
{
    if (!c) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    SYNC_EXT(c);
    VoState h;
    init_state(c, &h);
    int rc = write_state(c, &h);
    if (rc) return rc;
    VoExt e;
    std::memset(&e, 0, sizeof(e));
    for (int i = 0; i < VO_EXT_RING; ++i) { e.slot[i] = -1; e.status[i] = VO_STATUS_OK; }
    HIPCHK(hipMemcpyAsync(c->d.ext, &e, sizeof(e), hipMemcpyHostToDevice, c->s));
    HIPCHK(hipMemsetAsync(c->d.hist, 0, sizeof(uint32_t) * VO_HIST_BINS, c->s));
    for (int q = 1; q < VO_EXT_QUEUES; ++q)
        HIPCHK(hipMemsetAsync(c->xs[q].hist, 0, sizeof(uint32_t) * VO_HIST_BINS, c->s));
    c->fidx = 0;
    c->ext_ready = 0;
    HIPCHK(hipMemsetAsync(c->d.ctr, 0, sizeof(unsigned) * VO_CTR_WORDS, c->s));   // + frame counters
    vo::launch_frame_begin(c->d, VO_MODE_FRAME, c->s);     // frame 0 set up on the device
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->s));
    return VO_OK;
}

int vo_set_ground_truth(vo_ctx* c, const double* poses12, int n)
{
    if (!c || n < 0 || (n > 0 && !poses12)) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    HIPCHK(hipStreamSynchronize(c->s));
    if (n > c->gt_cap) {
        if (c->d.gt) (void)hipFree((void*)c->d.gt);
        double* g = nullptr;
        HIPCHK(hipMalloc((void**)&g, sizeof(double) * 12 * (size_t)n));
        c->d.gt = g;
        c->gt_cap = n;
    }
    if (n) HIPCHK(hipMemcpy((void*)c->d.gt, poses12, sizeof(double) * 12 * (size_t)n, hipMemcpyHostToDevice));
    c->d.gt_n = n;
    return VO_OK;
}

int vo_extract(vo_ctx* c, const uint8_t* gray, size_t stride, vo_kp* kps, uint64_t* desc, int* n, uint8_t* blurred)
{
    if (!c || !gray || !n) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    int rc = upload_frame(c, gray, stride, c->s);
    if (rc) return rc;
    enqueue_extract(c, c->d.frame_in, 0);      // slot VO_STAGE_SLOT: the trajectory's slots are untouched
    HIPCHK(hipGetLastError());
    VoExt e;
    rc = read_ext(c, &e);
    if (rc) return rc;
    if (e.stage_status != VO_STATUS_OK) return VO_ERR_CAPACITY;
    const int nk = e.n_kps[VO_STAGE_SLOT];
    *n = nk;
    if (kps && nk) HIPCHK(hipMemcpy(kps, c->d.kps[VO_STAGE_SLOT], sizeof(vo_kp) * nk, hipMemcpyDeviceToHost));
    if (desc && nk)
        HIPCHK(hipMemcpy(desc, c->d.desc[VO_STAGE_SLOT], sizeof(uint64_t) * 8 * nk, hipMemcpyDeviceToHost));
    if (blurred)
        HIPCHK(hipMemcpy(blurred, c->d.blurred, (size_t)c->cfg.width * c->cfg.height, hipMemcpyDeviceToHost));
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
    vo::launch_stencil(c->d, c->d.frame_in, 1, c->s);
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
    SYNC_EXT(c);
    HIPCHK(hipStreamSynchronize(c->s));
    const int a = VO_STAGE_SLOT, b = VO_STAGE_SLOT + 1;     // stage slots: the trajectory's stay intact
    HIPCHK(hipMemcpy(c->d.desc[a], d_prev, sizeof(uint64_t) * 8 * n_prev, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d.desc[b], d_cur, sizeof(uint64_t) * 8 * n_cur, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d.pre[a], p0.data(), sizeof(uint32_t) * n_prev, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d.pre[b], p1.data(), sizeof(uint32_t) * n_cur, hipMemcpyHostToDevice));
    const int nk2[2] = {n_prev, n_cur};
    HIPCHK(hipMemcpy(c->d.ext->n_kps + a, nk2, sizeof(nk2), hipMemcpyHostToDevice));
    VoState h;
    int rc = read_state(c, &h);
    if (rc) return rc;
    VoState saved = h;
    h.prev = a; h.cur = b;
    h.status = VO_STATUS_OK; h.mode = VO_MODE_STAGE;
    rc = write_state(c, &h);
    if (rc) return rc;
    vo::launch_match(c->d, c->s);
    HIPCHK(hipGetLastError());
    rc = read_state(c, &h);
    if (rc) return rc;
    *m = h.M;
    if (out && h.M) HIPCHK(hipMemcpy(out, c->d.match_pairs, sizeof(vo_match_t) * h.M, hipMemcpyDeviceToHost));
    // restore the trajectory bookkeeping (stage calls do not advance the loop)
    return restore_state(c, &saved);
}

int vo_ransac_F(vo_ctx* c, const double* pts, int m, uint64_t seed, double F[9], int* fitted, int32_t* inlier_idx,
                int* n_inl, int* best_k, int* n_evaluated, int32_t* counts)
{
    if (!c || !pts || m < 8 || m > c->cfg.max_kpts) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    HIPCHK(hipStreamSynchronize(c->s));
    HIPCHK(hipMemcpy(c->d.pts, pts, sizeof(double) * 4 * (size_t)m, hipMemcpyHostToDevice));
    VoState h;
    int rc = read_state(c, &h);
    if (rc) return rc;
    VoState saved = h;
    h.status = VO_STATUS_OK; h.mode = VO_MODE_STAGE;
    h.M = m; h.scored = (m / c->cfg.ransac_chunk_threads) * c->cfg.ransac_chunk_threads;
    h.frame_seed = seed; h.bestk = -1; h.need_more = 0; h.fitted = 0; h.n_inl = 0;
    rc = write_state(c, &h);
    if (rc) return rc;
    vo::launch_ransac(c->d, c->max_hyp, c->s);
    vo::launch_refit(c->d, 0, c->s);
    HIPCHK(hipGetLastError());
    rc = read_state(c, &h);
    if (rc) return rc;
    if (F) std::memcpy(F, h.model_F, sizeof(h.model_F));
    if (fitted) *fitted = h.fitted;
    if (n_inl) *n_inl = h.n_inl;
    if (best_k) *best_k = h.bestk;
    if (n_evaluated) *n_evaluated = h.n_eval;
    if (inlier_idx && h.bestk >= 0 && h.n_inl > 0)
        HIPCHK(hipMemcpy(inlier_idx, c->d.inl, sizeof(int32_t) * h.n_inl, hipMemcpyDeviceToHost));
    if (counts && h.n_eval > 0)
        HIPCHK(hipMemcpy(counts, c->d.counts, sizeof(int32_t) * std::min(h.n_eval, VO_MAX_HYP), hipMemcpyDeviceToHost));
    // the model (F + inliers) persists like FundamentalMatrix model (VisualOdometry.cpp:49)
    saved.model_n = h.model_n;
    std::memcpy(saved.model_F, h.model_F, sizeof(h.model_F));
    return restore_state(c, &saved);
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
    HIPCHK(hipStreamSynchronize(c->s));
    HIPCHK(hipMemcpy(c->d.model_p, mp.data(), sizeof(float) * mp.size(), hipMemcpyHostToDevice));
    VoState h;
    int rc = read_state(c, &h);
    if (rc) return rc;
    VoState saved = h;
    h.status = VO_STATUS_OK; h.mode = VO_MODE_STAGE;
    h.model_n = n;
    std::memcpy(h.model_F, F, sizeof(h.model_F));
    h.scale_override = scale;
    rc = write_state(c, &h);
    if (rc) return rc;
    vo::launch_pose_prep(c->d, c->s);
    vo::launch_triangulate(c->d, c->s);
    HIPCHK(hipGetLastError());
    rc = read_state(c, &h);
    if (rc) return rc;
    int ret = VO_OK;
    if (h.status == VO_STATUS_DEGENERATE) ret = VO_ERR_DEGENERATE_E;
    else if (h.status != VO_STATUS_OK) ret = VO_ERR_STATE;
    if (ret == VO_OK) {
        if (R) std::memcpy(R, h.pose_R, sizeof(h.pose_R));
        if (t) std::memcpy(t, h.pose_t, sizeof(h.pose_t));
    }
    if (counts4) std::memcpy(counts4, h.counts4, sizeof(h.counts4));
    rc = restore_state(c, &saved);
    return ret != VO_OK ? ret : rc;
}

int vo_process_frame(vo_ctx* c, const uint8_t* gray, size_t stride, double pose_out[12], int* status, int32_t* info)
{
    if (!c) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    if (gray) {
        int rc = upload_frame(c, gray, stride, c->serial ? c->s : c->se[c->fidx % VO_EXT_QUEUES]);
        if (rc) return rc;
    }
    enqueue_frame(c, gray ? c->d.frame_in : nullptr, c->out_dev, nullptr, false);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(c->out_host, c->out_dev, sizeof(VoFrameOut), hipMemcpyDeviceToHost, c->s));
    HIPCHK(hipStreamSynchronize(c->s));
    const VoFrameOut& o = c->out_host[0];
    if (pose_out) std::memcpy(pose_out, o.pose, sizeof(o.pose));
    if (status) *status = o.status;
    if (info) {
        info[0] = o.n_kps; info[1] = o.n_matches; info[2] = o.n_inl; info[3] = o.best_k;
        info[4] = o.n_eval; info[5] = o.fitted; info[6] = 0; info[7] = 0;
    }
    return o.status == VO_STATUS_DEGENERATE ? VO_ERR_DEGENERATE_E : VO_OK;
}

int vo_process_frames_device(vo_ctx* c, const uint8_t* d_frames, size_t frame_bytes, int nframes, double* poses_out,
                             int* status_out, int32_t* info_out)
{
    if (!c || !d_frames || nframes < 0) return VO_ERR_ARG;
    if (frame_bytes < (size_t)c->cfg.width * c->cfg.height) return VO_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    int rc = ensure_out(c, std::max(nframes, 1));
    if (rc) return rc;
    EvRec rec{&c->ev_pool, 0, c->timing >= 100 ? c->timing - 100 : -1, 0, {}};
    EvRec* evp = c->timing ? &rec : nullptr;
    for (int f = 0; f < nframes; ++f)
        enqueue_frame(c, d_frames + (size_t)f * frame_bytes, c->out_dev + f, evp, f + 1 < nframes);
    HIPCHK(hipGetLastError());
    if (nframes)
        HIPCHK(hipMemcpyAsync(c->out_host, c->out_dev, sizeof(VoFrameOut) * nframes, hipMemcpyDeviceToHost, c->s));
    HIPCHK(hipStreamSynchronize(c->s));
    if (evp) {
        const int nk = vo::kernel_count();
        c->ktime_ms.assign(nk, 0.f);
        c->kcount.assign(nk, 0);
        for (const auto& sp : rec.spans) {
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, c->ev_pool[sp.second], c->ev_pool[sp.second + 1]);
            c->ktime_ms[sp.first] += ms;
            c->kcount[sp.first] += 1;
        }
    }
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
    if (!c) return VO_ERR_ARG;
    int nk = std::min<int>((int)c->ktime_ms.size(), cap);
    for (int k = 0; k < nk; ++k) {
        if (names) names[k] = vo::kernel_name(k);
        if (ms) ms[k] = c->kcount[k] ? c->ktime_ms[k] / (float)c->kcount[k] : -1.f;
    }
    return nk;
}

// diagnostics: copy the stamp buffer (VO_STAMPS builds; returns 0 entries otherwise)
int vo_debug_stamps(vo_ctx* c, unsigned long long* out, int n)
{
    if (!c || !c->d.dbg) return 0;
    int m = std::min(n, c->max_hyp * 16);
    HIPCHK(hipStreamSynchronize(c->s));
    HIPCHK(hipMemcpy(out, c->d.dbg, sizeof(unsigned long long) * m, hipMemcpyDeviceToHost));
    return m;
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
