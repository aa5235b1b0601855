// minehip.cpp -- C-ABI of libminehip.so (declared in include/minehip.h).
//
// Per device: one HIP stream, a partials buffer, a 16-byte running minimum
// and a pinned 16-byte host slot, created on first use and reused by every
// call.  A search enqueues all of its launches (fast runs, generic edges,
// merges) on that stream and synchronises once, when it copies the 16-byte
// result back.  No CPU fallback exists: without a gfx950 device the calls fail
// with MH_ENODEV.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/minehip.h"
#include "../../include/minehip_server.h"
#include "layout.hpp"
#include "multi.hpp"
#include "plan.hpp"
#include "sched.hpp"

namespace mh {
hipError_t fast_module_init(int dev);
hipError_t launch_fast(int dev, int J, int mode, const FastArgs& a, Partial* partials, hipStream_t s);
hipError_t launch_generic_scan(const GenArgs& a, Partial* partials, uint32_t blocks, hipStream_t s);
hipError_t launch_hash_batch(const GenArgs& a, const uint64_t* d_nonces, uint64_t* d_out, uint64_t n,
                             hipStream_t s);
hipError_t launch_merge(const Partial* partials, uint32_t n, Partial* best, hipStream_t s);
}  // namespace mh

namespace {

using mh::Partial;

thread_local std::string g_err;

int fail(int code, const std::string& what) {
    g_err = what;
    return code;
}

}  // namespace

namespace mh {
int set_error(int code, const char* what) { return fail(code, what); }
}  // namespace mh

namespace {

#define MH_HIP(call)                                                                                 \
    do {                                                                                             \
        hipError_t e_ = (call);                                                                      \
        if (e_ != hipSuccess) return fail(MH_EHIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

constexpr uint64_t kBatchChunk = 1u << 22;  // nonces per hash_batch transfer
constexpr int kEventPairs = 512;             // profiled launches buffered before harvesting
constexpr uint32_t kQueueSlots = 4096;       // work-queue counters per search (one per fast launch)

struct Timed {
    hipEvent_t start = nullptr, stop = nullptr;
    int kind;  // 0 fast, 1 generic
    int var;   // fast: kernel variant and lane length, var_index(J, mode, L)
};

// per fast_search<J, MODE> variant: launches, nonces, ns, algorithmic instructions
struct VarStat {
    uint64_t launches = 0, nonces = 0, ns = 0, ops = 0, slots = 0;
};
constexpr int kVariants = 16 * mh::kModes * 5;  // J < 16, mode < kModes, L = 1..5
inline int var_index(int J, int mode, int L) { return J + 16 * mode + 16 * mh::kModes * (L - 1); }

struct DevCtx {
    std::mutex mu;
    int dev = -1;
    bool ready = false;
    hipStream_t stream = nullptr;              // every search's merge and copy; pieces with streams = 1
    // streams = 2: the pieces' streams, by priority: [0] coarse pieces (high), [1] the other pieces (low)
    hipStream_t ps[2] = {nullptr, nullptr};
    hipEvent_t ev_piece[2] = {nullptr, nullptr};  // each piece stream's work so far
    hipEvent_t ev_main = nullptr;                          // the main stream's (reset / merge)
    Partial* d_partials = nullptr;
    Partial* d_best = nullptr;
    Partial* h_best = nullptr;  // pinned
    uint64_t* d_nonces = nullptr;
    uint64_t* d_hashes = nullptr;
    uint32_t poff = 0;  // partials written since the last merge
    uint32_t* d_counters = nullptr;  // work-queue counters, zeroed at each search's start
    uint32_t qoff = 0;               // counters used by this search
    // profiling
    bool prof = false;
    std::vector<Timed> pool;
    int used = 0;
    uint64_t cnt[8] = {0};
    VarStat var[kVariants];
};

std::mutex g_tab_mu;
std::vector<std::unique_ptr<DevCtx>> g_tab;
int g_ndev = -1;

int device_count_impl() {
    std::lock_guard<std::mutex> lk(g_tab_mu);
    if (g_ndev < 0) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
        g_ndev = n;
        g_tab.resize((size_t)n);
        for (auto& p : g_tab) p.reset(new DevCtx());
    }
    return g_ndev;
}

// Returns the context for dev, initialised, with its mutex NOT held.
int get_ctx(int dev, DevCtx** out) {
    const int n = device_count_impl();
    if (n <= 0) return fail(MH_ENODEV, "no HIP device visible");
    if (dev < 0 || dev >= n) return fail(MH_EINVAL, "device index out of range");
    DevCtx* c = g_tab[(size_t)dev].get();
    *out = c;
    return MH_OK;
}

int init_locked(DevCtx* c, int dev) {
    if (c->ready) return MH_OK;
    MH_HIP(hipSetDevice(dev));
    hipDeviceProp_t prop;
    MH_HIP(hipGetDeviceProperties(&prop, dev));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(MH_ENODEV, std::string("device is ") + prop.gcnArchName + ", kernels are built for gfx950 only");
    // each resource only once: a call after a failed init (e.g. the code object
    // did not load) resumes where that one stopped instead of allocating again
    if (!c->stream) MH_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    if (!c->ps[0] || !c->ps[1]) {
        int least = 0, greatest = 0;
        MH_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));  // gfx950: 1 .. -1
        if (!c->ps[0]) MH_HIP(hipStreamCreateWithPriority(&c->ps[0], hipStreamNonBlocking, greatest));
        if (!c->ps[1]) MH_HIP(hipStreamCreateWithPriority(&c->ps[1], hipStreamNonBlocking, least));
    }
    for (auto& e : c->ev_piece)
        if (!e) MH_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (!c->ev_main) MH_HIP(hipEventCreateWithFlags(&c->ev_main, hipEventDisableTiming));
    if (!c->d_partials) MH_HIP(hipMalloc(&c->d_partials, sizeof(Partial) * mh::kMaxBlocksPerLaunch));
    if (!c->d_best) MH_HIP(hipMalloc(&c->d_best, sizeof(Partial)));
    if (!c->d_counters) MH_HIP(hipMalloc(&c->d_counters, sizeof(uint32_t) * kQueueSlots));
    if (!c->h_best) MH_HIP(hipHostMalloc(&c->h_best, sizeof(Partial), hipHostMallocDefault));
    if (!c->d_nonces) MH_HIP(hipMalloc(&c->d_nonces, sizeof(uint64_t) * kBatchChunk));
    if (!c->d_hashes) MH_HIP(hipMalloc(&c->d_hashes, sizeof(uint64_t) * kBatchChunk));
    if (c->pool.empty()) c->pool.resize(kEventPairs);
    for (auto& t : c->pool) {
        if (!t.start) MH_HIP(hipEventCreate(&t.start));
        if (!t.stop) MH_HIP(hipEventCreate(&t.stop));
    }
    MH_HIP(mh::fast_module_init(dev));  // the fast_search code object (issue-priority build)
    c->dev = dev;
    c->ready = true;
    return MH_OK;
}

// Stream must be idle or synchronised by the caller.
int harvest_locked(DevCtx* c) {
    for (int i = 0; i < c->used; ++i) {
        float ms = 0.f;
        MH_HIP(hipEventElapsedTime(&ms, c->pool[(size_t)i].start, c->pool[(size_t)i].stop));
        const uint64_t ns = (uint64_t)((double)ms * 1.0e6);
        c->cnt[c->pool[(size_t)i].kind == 0 ? 2 : 5] += ns;
        if (c->pool[(size_t)i].kind == 0) c->var[c->pool[(size_t)i].var].ns += ns;
    }
    c->used = 0;
    return MH_OK;
}

// The piece streams start after the main stream's work so far (the reset, a merge).
int piece_streams_wait_main(DevCtx* c) {
    MH_HIP(hipEventRecord(c->ev_main, c->stream));
    for (auto s : c->ps) MH_HIP(hipStreamWaitEvent(s, c->ev_main, 0));
    return MH_OK;
}

// Fold the pending partials into the running minimum.  With two piece
// streams the merge (on the main stream) first waits for both, and both wait
// for the merge before any later piece reuses the partials buffer.
int flush_partials(DevCtx* c, bool split) {
    if (!c->poff) return MH_OK;
    if (split) {
        for (int k = 0; k < 2; ++k) {
            MH_HIP(hipEventRecord(c->ev_piece[k], c->ps[k]));
            MH_HIP(hipStreamWaitEvent(c->stream, c->ev_piece[k], 0));
        }
    }
    MH_HIP(mh::launch_merge(c->d_partials, c->poff, c->d_best, c->stream));
    c->poff = 0;
    if (split) return piece_streams_wait_main(c);
    return MH_OK;
}

// Coarse pieces (the full L: 1,000-nonce lanes) go to the high-priority stream, the others
// (shorter lanes, generic edges, the tail split) to the low-priority one.
bool coarse_piece(const mh::Piece& p, const mh::PlanOpts& opt) { return p.kind == 0 && p.L == opt.lower_digits; }

// An Early piece (layout.hpp kMode*Early) enumerates its innermost digit and the L - 1 group digits
// before it inside word J: the kernel adds every group digit into word J, so a digit elsewhere
// would be hashed at the wrong place.  make_fast_args only builds such pieces; this re-checks it
// where a piece reaches the kernel, with the U digits' hole inside the d digits.
bool early_piece_ok(const mh::Piece& p) {
    const mh::FastArgs& a = p.fa;
    const uint32_t J = (uint32_t)p.J;
    if ((a.inner >> 2) != J || a.hole + a.hole_w > a.n_hi + a.L) return false;
    for (uint32_t j = 0; j + 1u < a.L; ++j) {
        const uint32_t pos = a.g_last - j - (j >= a.g_hole ? 1u : 0u);
        if (pos > a.g_last || (pos >> 2) != J) return false;
    }
    return true;
}

// Enqueue one piece on the context's stream.  Its workgroups write their
// partials after those of the previous pieces; one merge folds them all (or
// earlier, when the buffer would overflow), instead of one merge per piece.
int enqueue_piece(DevCtx* c, const mh::Piece& p, const mh::PlanOpts& opt, bool split) {
    hipStream_t s = !split ? c->stream : c->ps[coarse_piece(p, opt) ? 0 : 1];
    uint32_t blocks;
    if (p.kind == 0) {
        // host-side shape checks: the grid covers exactly n_runs lanes and the
        // partials buffer holds one slot per block
        if (p.fa.n_runs == 0 || p.fa.L < 1 || p.fa.L > 5 || p.fa.n_hi + p.fa.L > 20)
            return fail(MH_EINTERNAL, "internal: bad fast piece");
        if (p.fa.mode >= mh::kModeOneEarly && !early_piece_ok(p))
            return fail(MH_EINTERNAL, "internal: bad Early piece (an enumerated digit outside word J)");
        blocks = (p.fa.n_runs + mh::kBlockThreads - 1) / mh::kBlockThreads;
    } else {
        if (p.ga.count == 0 || p.ga.count > (uint64_t)mh::kMaxBlocksPerLaunch * mh::kBlockThreads)
            return fail(MH_EINTERNAL, "internal: bad generic piece");
        blocks = (uint32_t)((p.ga.count + mh::kBlockThreads - 1) / mh::kBlockThreads);
    }
    if (blocks > mh::kMaxBlocksPerLaunch) return fail(MH_EINTERNAL, "internal: grid too large");
    if (c->poff + blocks > mh::kMaxBlocksPerLaunch) {
        const int rc = flush_partials(c, split);
        if (rc) return rc;
    }
    Partial* out = c->d_partials + c->poff;
    Timed* tm = nullptr;
    mh::FastArgs fa = p.fa;
    if (p.kind == 0) {
        fa.n_chunks = blocks;
        // work queue while this search has counters left (a longer search runs the rest static)
        fa.counter = (opt.queue && c->qoff < kQueueSlots) ? c->d_counters + c->qoff++ : nullptr;
    }
    if (c->prof) {
        if (c->used == kEventPairs) {
            MH_HIP(hipStreamSynchronize(c->stream));
            for (auto ps : c->ps) MH_HIP(hipStreamSynchronize(ps));
            int rc = harvest_locked(c);
            if (rc) return rc;
        }
        tm = &c->pool[(size_t)c->used++];
        tm->kind = p.kind;
        tm->var = p.kind == 0 ? var_index(p.J, p.mode, p.L) : 0;
        MH_HIP(hipEventRecord(tm->start, s));
    }
    if (p.kind == 0)
        MH_HIP(mh::launch_fast(c->dev, p.J, p.mode, fa, out, s));
    else
        MH_HIP(mh::launch_generic_scan(p.ga, out, blocks, s));
    if (tm) MH_HIP(hipEventRecord(tm->stop, s));
    c->poff += blocks;
    if (c->prof) {
        if (p.kind == 0) {
            const uint64_t n = p.count;
            c->cnt[0] += 1;
            c->cnt[1] += n;
            c->cnt[3] += n * (uint64_t)p.ops;
            c->cnt[6] += n * (uint64_t)p.slots;
            VarStat& v = c->var[var_index(p.J, p.mode, p.L)];
            v.launches += 1;
            v.nonces += n;
            v.ops += n * (uint64_t)p.ops;
            v.slots += n * (uint64_t)p.slots;
        } else {
            c->cnt[4] += p.count;
        }
    }
    return MH_OK;
}

// Planner knobs, overridable for tests and tuning (the result never depends
// on them -- tests/test_gpu_parity.py checks exactly that):
//   MINEHIP_LOWER_DIGITS   L, digits enumerated inside one lane (1..5, default 3)
//   MINEHIP_MIN_LANES      lower L per bucket until it has this many runs (2^19)
//   MINEHIP_LAUNCH_NONCES  nonces per fast launch (default 2^35)
//   MINEHIP_GENERIC_BELOW  buckets with fewer nonces go to the generic kernel (2^20)
//   MINEHIP_MAX_BLOCKS     workgroups per launch (1..kMaxBlocksPerLaunch)
//   MINEHIP_STREAMS        1: one stream; 2: coarse / fine pieces on high / low priority
//                          streams (default 2)
//   MINEHIP_FINE_TAIL      nonces at the end of each full-L bucket planned at L - 1 (default
//                          2^28; 0: none)
//   MINEHIP_QUEUE          1: fast launches as work queues (workgroups claim chunks, so faster
//                          XCDs take more; default); 0: one workgroup per chunk
//   MINEHIP_EARLY          1: the Early layouts where a nonce costs less with the digit ending the
//                          word before the last digit's innermost (default); 0: never
mh::PlanOpts plan_opts() {
    mh::PlanOpts o;
    if (const char* e = getenv("MINEHIP_LOWER_DIGITS")) {
        const int v = atoi(e);
        if (v >= 1 && v <= 5) o.lower_digits = v;
    }
    if (const char* e = getenv("MINEHIP_MIN_LANES")) o.min_lanes = strtoull(e, nullptr, 10);
    if (const char* e = getenv("MINEHIP_LAUNCH_NONCES")) {
        const unsigned long long v = strtoull(e, nullptr, 10);
        if (v >= 1) o.max_nonces_per_launch = v;
    }
    if (const char* e = getenv("MINEHIP_GENERIC_BELOW")) o.generic_below = strtoull(e, nullptr, 10);
    if (const char* e = getenv("MINEHIP_MAX_BLOCKS")) {
        const unsigned long long v = strtoull(e, nullptr, 10);
        if (v >= 1 && v <= mh::kMaxBlocksPerLaunch) o.max_blocks = (uint32_t)v;
    }
    if (const char* e = getenv("MINEHIP_STREAMS")) {
        const int v = atoi(e);
        if (v == 1 || v == 2) o.streams = v;
    }
    if (const char* e = getenv("MINEHIP_FINE_TAIL")) o.fine_tail = strtoull(e, nullptr, 10);
    if (const char* e = getenv("MINEHIP_QUEUE")) {
        const int v = atoi(e);
        if (v == 0 || v == 1) o.queue = v;
    }
    if (const char* e = getenv("MINEHIP_EARLY")) {
        const int v = atoi(e);
        if (v == 0 || v == 1) o.early = v;
    }
    return o;
}

uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// busy_ns (optional): the search's own wall time, from holding the initialised device to having
// its result -- without the wait for another thread's search on the same device.
int search_impl(int dev, const mh::Prefix& pre, uint64_t lower, uint64_t upper, uint64_t* oh, uint64_t* on,
                uint64_t* busy_ns = nullptr) {
    DevCtx* c;
    int rc = get_ctx(dev, &c);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(c->mu);
    rc = init_locked(c, dev);
    if (rc) return rc;
    const uint64_t t0 = now_ns();
    MH_HIP(hipSetDevice(dev));
    MH_HIP(hipMemsetAsync(c->d_best, 0xFF, sizeof(Partial), c->stream));
    const mh::PlanOpts opt = plan_opts();
    if (opt.queue) MH_HIP(hipMemsetAsync(c->d_counters, 0, sizeof(uint32_t) * kQueueSlots, c->stream));
    c->qoff = 0;
    // Two streams only when there is something to overlap: coarse pieces and others.  A small
    // search (generic edges, short-lane buckets) stays on one stream and skips the events.  The
    // plan is streamed, never stored (a range can hold ~2^30 pieces); this first pass stops as
    // soon as it has seen both kinds.
    bool any_coarse = false, any_fine = false;
    if (opt.streams == 2)
        mh::plan_search(pre, lower, upper, opt, [&](const mh::Piece& p) {
            (coarse_piece(p, opt) ? any_coarse : any_fine) = true;
            return !(any_coarse && any_fine);
        });
    const bool split = opt.streams == 2 && any_coarse && any_fine;
    if (split) {  // the piece streams start after the reset (and after the previous search)
        rc = piece_streams_wait_main(c);
        if (rc) return rc;
    }
    int err = MH_OK;
    c->poff = 0;
    mh::plan_search(pre, lower, upper, opt, [&](const mh::Piece& p) {
        err = enqueue_piece(c, p, opt, split);
        return err == MH_OK;
    });
    if (!err) err = flush_partials(c, split);
    if (err) {
        for (auto ps : c->ps)
            if (ps) (void)hipStreamSynchronize(ps);
        (void)hipStreamSynchronize(c->stream);
        return err;
    }
    MH_HIP(hipMemcpyAsync(c->h_best, c->d_best, sizeof(Partial), hipMemcpyDeviceToHost, c->stream));
    MH_HIP(hipStreamSynchronize(c->stream));
    if (c->prof) {
        rc = harvest_locked(c);
        if (rc) return rc;
    }
    *oh = c->h_best->hash;
    *on = c->h_best->nonce;
    if (busy_ns) *busy_ns = now_ns() - t0;
    return MH_OK;
}

int check_common(const uint8_t* msg, size_t len) {
    if (msg == nullptr && len != 0) return fail(MH_EINVAL, "msg is NULL");
    if (len > MH_MAX_MSG_LEN) return fail(MH_ETOOLONG, "message longer than MH_MAX_MSG_LEN");
    return MH_OK;
}

}  // namespace

extern "C" {

int mh_abi_version(void) { return MH_ABI_VERSION; }

int mh_device_count(void) { return device_count_impl(); }

const char* mh_last_error(void) { return g_err.c_str(); }

int mh_search(int dev, const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper, uint64_t* out_hash,
              uint64_t* out_nonce) {
    g_err.clear();
    if (!out_hash || !out_nonce) return fail(MH_EINVAL, "NULL output pointer");
    int rc = check_common(msg, len);
    if (rc) return rc;
    if (lower > upper) return fail(MH_ERANGE, "lower > upper");
    mh::Prefix pre;
    mh::absorb_prefix(msg, len, &pre);
    return search_impl(dev, pre, lower, upper, out_hash, out_nonce);
}

int mh_search_multi(const int* devs, int ndev, const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper,
                    uint64_t chunk, uint64_t* out_hash, uint64_t* out_nonce) {
    g_err.clear();
    if (!out_hash || !out_nonce || !devs || ndev <= 0) return fail(MH_EINVAL, "bad arguments");
    if (ndev > MH_MAX_WORKERS) return fail(MH_EINVAL, "more than MH_MAX_WORKERS devices listed");
    int rc = check_common(msg, len);
    if (rc) return rc;
    if (lower > upper) return fail(MH_ERANGE, "lower > upper");
    const int n = mh_device_count();
    for (int i = 0; i < ndev; ++i)
        if (devs[i] < 0 || devs[i] >= n) return fail(n <= 0 ? MH_ENODEV : MH_EINVAL, "device index out of range");
    mh::Prefix pre;
    mh::absorb_prefix(msg, len, &pre);
    // One device and adaptive chunks: nothing to balance, so one search (one
    // plan, full-size launches) instead of a chain of shrinking chunks.
    // test hook of the dev build only (`make dev`, -DMH_DEV_HOOKS):
    // MINEHIP_TEST_FAIL_WORKER=i makes worker i's first search fail with
    // MH_EHIP, to exercise the hand-back path on a one-GPU box
    int fail_worker = -1;
    // MINEHIP_TEST_SPAWN_LIMIT=k (dev build only): the host thread of every worker after the first
    // k fails to start (std::system_error, as when the process is out of threads), so the
    // start-failure path of both coordinators runs on any box
    mh::ThreadStart start;
#ifdef MH_DEV_HOOKS
    if (const char* e = getenv("MINEHIP_TEST_FAIL_WORKER")) fail_worker = atoi(e);
    if (const char* e = getenv("MINEHIP_TEST_SPAWN_LIMIT")) {
        auto started = std::make_shared<std::atomic<int>>(0);
        const int limit = atoi(e);
        start = [started, limit](std::function<void()> fn) {
            if ((*started)++ >= limit)
                throw std::system_error(std::make_error_code(std::errc::resource_unavailable_try_again));
            return std::thread(std::move(fn));
        };
    }
#endif
    if (ndev == 1 && chunk == 0 && fail_worker < 0 && !start)
        return search_impl(devs[0], pre, lower, upper, out_hash, out_nonce);
    // Adaptive: one rate-weighted shard per device (+ a short dynamic tail on long ranges), multi.hpp.
    if (chunk == 0) {
        const mh::SpanSearch search = [&](int worker, int dev, uint64_t lo, uint64_t hi, uint64_t* h, uint64_t* n,
                                          uint64_t* ns, std::string* err) {
            const int r = (worker == fail_worker) ? fail(MH_EHIP, "injected failure (dev build test hook)")
                                                  : search_impl(dev, pre, lo, hi, h, n, ns);
            if (r) *err = g_err;  // this worker thread's description
            return r;
        };
        std::string err;
        const int r = mh::search_shards(devs, ndev, pre, lower, upper, plan_opts(), search, out_hash, out_nonce, &err,
                                        start);
        return r ? fail(r, err) : MH_OK;
    }
    // Fixed chunks: one miner per listed device, fed by the server's scheduler (sched.hpp) with
    // chunks of exactly `chunk` nonces (multi.cpp search_chunks).  A device that fails hands its
    // chunk back to the others.
    const mh::ChunkSearch csearch = [&](int worker, uint64_t lo, uint64_t hi, uint64_t* h, uint64_t* nn,
                                        std::string* err) {
        const int r = (worker == fail_worker) ? fail(MH_EHIP, "injected failure (dev build test hook)")
                                              : search_impl(devs[worker], pre, lo, hi, h, nn);
        if (r) *err = g_err;
        return r;
    };
    std::string err;
    const int r = mh::search_chunks(ndev, msg, len, lower, upper, chunk, csearch, out_hash, out_nonce, &err, start);
    return r ? fail(r, err) : MH_OK;
}

int mh_hash_batch(int dev, const uint8_t* msg, size_t len, const uint64_t* nonces, size_t n, uint64_t* out_hashes) {
    g_err.clear();
    int rc = check_common(msg, len);
    if (rc) return rc;
    if (n == 0) return MH_OK;
    if (!nonces || !out_hashes) return fail(MH_EINVAL, "NULL buffer");
    DevCtx* c;
    rc = get_ctx(dev, &c);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(c->mu);
    rc = init_locked(c, dev);
    if (rc) return rc;
    MH_HIP(hipSetDevice(dev));
    mh::Prefix pre;
    mh::absorb_prefix(msg, len, &pre);
    mh::GenArgs ga;
    mh::make_gen_args(pre, &ga);
    for (size_t off = 0; off < n; off += kBatchChunk) {
        const size_t m = (n - off < kBatchChunk) ? n - off : kBatchChunk;
        MH_HIP(hipMemcpyAsync(c->d_nonces, nonces + off, m * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
        MH_HIP(mh::launch_hash_batch(ga, c->d_nonces, c->d_hashes, m, c->stream));
        MH_HIP(hipMemcpyAsync(out_hashes + off, c->d_hashes, m * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
        MH_HIP(hipStreamSynchronize(c->stream));
    }
    return MH_OK;
}

int mh_profile_enable(int dev, int on) {
    g_err.clear();
    DevCtx* c;
    int rc = get_ctx(dev, &c);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(c->mu);
    rc = init_locked(c, dev);
    if (rc) return rc;
    MH_HIP(hipStreamSynchronize(c->stream));
    rc = harvest_locked(c);  // timings of launches already recorded stay counted
    if (rc) return rc;
    if (on) {  // enabling starts a fresh count; disabling keeps the counts readable
        memset(c->cnt, 0, sizeof c->cnt);
        for (auto& v : c->var) v = VarStat();
    }
    c->prof = on != 0;
    return MH_OK;
}

int mh_profile_read(int dev, uint64_t* out, int n) {
    g_err.clear();
    if (!out || n < 0) return fail(MH_EINVAL, "bad arguments");
    DevCtx* c;
    int rc = get_ctx(dev, &c);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->ready) {
        MH_HIP(hipStreamSynchronize(c->stream));
        rc = harvest_locked(c);
        if (rc) return rc;
    }
    for (int i = 0; i < n && i < 8; ++i) out[i] = c->cnt[i];
    return MH_OK;
}

int mh_profile_kernels(int dev, mh_kernel_stat* out, int cap) {
    g_err.clear();
    if (cap < 0 || (!out && cap > 0)) return fail(MH_EINVAL, "bad arguments");
    DevCtx* c;
    int rc = get_ctx(dev, &c);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->ready) {
        MH_HIP(hipStreamSynchronize(c->stream));
        rc = harvest_locked(c);
        if (rc) return rc;
    }
    int n = 0;
    for (int i = 0; i < kVariants; ++i) {
        const VarStat& v = c->var[i];
        if (!v.launches) continue;
        if (n < cap) {
            out[n].word = i % 16;
            out[n].mode = (i / 16) % mh::kModes;
            out[n].lo_digits = i / (16 * mh::kModes) + 1;
            out[n].reserved = 0;
            out[n].launches = v.launches;
            out[n].nonces = v.nonces;
            out[n].ns = v.ns;
            out[n].ops = v.ops;
            out[n].slots = v.slots;
        }
        ++n;
    }
    return n;
}

int64_t mh_plan(const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper, mh_piece* out, int64_t cap) {
    g_err.clear();
    int rc = check_common(msg, len);
    if (rc) return rc;
    if (lower > upper) return fail(MH_ERANGE, "lower > upper");
    if (cap < 0) return fail(MH_EINVAL, "cap < 0");
    mh::Prefix pre;
    mh::absorb_prefix(msg, len, &pre);
    int64_t k = 0;
    const mh::PlanOpts opt = plan_opts();
    mh::plan_search(pre, lower, upper, opt, [&](const mh::Piece& p) {
        if (k >= cap) {
            ++k;  // cap + 1 signals truncation
            return false;
        }
        if (out) {
            mh_piece& q = out[k];
            q.first = p.first;
            q.count = p.count;
            q.kind = p.kind;
            q.digits = p.digits;
            q.lo_digits = p.L;
            q.word = p.J;
            q.mode = p.mode;
            q.blocks = p.blocks;
            q.nonce_ops = p.ops;
            q.nonce_slots = p.slots;
        }
        ++k;
        return true;
    });
    return k;
}

int64_t mh_multi_plan(const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper, const double* weights,
                      int ndev, mh_span* out, int64_t cap) {
    g_err.clear();
    int rc = check_common(msg, len);
    if (rc) return rc;
    if (lower > upper) return fail(MH_ERANGE, "lower > upper");
    if (ndev <= 0 || ndev > MH_MAX_WORKERS || cap < 0) return fail(MH_EINVAL, "bad arguments");
    std::vector<double> w((size_t)ndev, 1.0);
    if (weights)
        for (int i = 0; i < ndev; ++i) {
            if (!(weights[i] > 0.0) || !std::isfinite(weights[i])) return fail(MH_EINVAL, "weights must be finite and > 0");
            w[(size_t)i] = weights[i];
        }
    mh::Prefix pre;
    mh::absorb_prefix(msg, len, &pre);
    mh::MultiPlan mp;
    mh::multi_plan(pre, lower, upper, plan_opts(), w, &mp);
    int64_t k = 0;
    auto put = [&](const mh::Span& s, int worker, int kind) {
        if (k < cap && out) {
            out[k].lower = s.lo;
            out[k].upper = s.hi;
            out[k].worker = worker;
            out[k].kind = kind;
            out[k].cost = mh::segments_cost(mp.segs, s.lo, s.hi);
        }
        ++k;
    };
    for (int i = 0; i < ndev; ++i)
        if (!mp.head[(size_t)i].empty) put(mp.head[(size_t)i], i, 0);
    for (const auto& s : mp.tail) put(s, -1, 1);
    return k;
}

int mh_multi_rates(const int* devs, int ndev, double* out) {
    g_err.clear();
    if (ndev < 0 || (ndev > 0 && (!devs || !out))) return fail(MH_EINVAL, "bad arguments");
    for (int i = 0; i < ndev; ++i) out[i] = mh::device_rate(devs[i]);
    return MH_OK;
}

}  // extern "C"
