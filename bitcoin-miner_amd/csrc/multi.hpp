// multi.hpp -- how mh_search_multi (chunk = 0) spreads one range over several devices
// (DESIGN.md §7).  Host only: the searches themselves are injected (SpanSearch), so the
// coordination runs under ThreadSanitizer without a GPU (tests/host/tsan_multi.cpp).
//
// Each worker (one listed device) gets ONE contiguous head shard up front, sized in proportion to
// its device's measured rate, so a step of the multi-GPU search is one search per device: one
// plan, full-size launches, one drain, one sync.  A range large enough that a few percent of it
// still makes long chunks (>= 2^35 nonces per worker, ~0.6 s) keeps its last 1/16 back as 2
// chunks per worker, handed out as the heads finish, which absorbs a device running slower than
// its rate predicted.  Rates persist per process, in cost units per ns (plan.hpp CostSeg: issue
// slots), so a shard holding short-lane buckets or generic edges does not make its device look
// slow.  Before any rate is known the shards are equal by cost.  A worker whose search fails
// hands its span back, cut for the workers still running.
#pragma once
#include <stdint.h>

#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "plan.hpp"

namespace mh {

constexpr uint64_t kTailMinPerWorker = 1ull << 35;  // nonces per worker before a dynamic tail is cut
constexpr int kTailDiv = 16;                         // the tail is 1/kTailDiv of the cost
constexpr uint64_t kRateMinNonces = 1ull << 30;      // shorter searches are latency, not rate
constexpr double kRateMaxUnsteady = 0.01;            // ... and spans of small buckets are off the model

struct MultiPlan {
    std::vector<CostSeg> segs;
    std::vector<Span> head;  // one per worker (may be empty)
    std::vector<Span> tail;  // non-empty, in nonce order
};

// The split of [lower, upper] over workers with rates in proportion to w (> 0).
void multi_plan(const Prefix& pre, uint64_t lower, uint64_t upper, const PlanOpts& opt,
                const std::vector<double>& w, MultiPlan* mp);

// The per-process rate table (slots per ns per device, 0 = not measured).
std::vector<double> worker_weights(const int* devs, int ndev);  // unknown rates: the mean of the known
void record_rate(int dev, double slots, uint64_t ns);            // EWMA
double device_rate(int dev);

// One search of [lo, hi] by `worker` on device `dev`: fills the (hash, nonce) minimum and the
// search's own busy time, or returns an MH_E* code with *err describing it.
using SpanSearch = std::function<int(int worker, int dev, uint64_t lo, uint64_t hi, uint64_t* hash,
                                     uint64_t* nonce, uint64_t* busy_ns, std::string* err)>;

// Starts one worker's host thread (std::thread by default).  May throw, as std::thread's
// constructor does when the process is out of threads; the dev build's MINEHIP_TEST_SPAWN_LIMIT
// and tests/host/tsan_multi.cpp inject a starter that throws after k threads.
using ThreadStart = std::function<std::thread(std::function<void()>)>;

// Runs the split with one host thread per worker.  MH_OK with the lexicographic minimum, or the
// first failure's code and text when every worker failed (some span was left unsearched).  Workers
// whose thread could not start leave their heads to the others.
int search_shards(const int* devs, int ndev, const Prefix& pre, uint64_t lower, uint64_t upper,
                  const PlanOpts& opt, const SpanSearch& search, uint64_t* out_hash, uint64_t* out_nonce,
                  std::string* err, const ThreadStart& start = {});

// One search of [lo, hi] by `worker` (the fixed-chunk path): the (hash, nonce) minimum, or an MH_E*
// code with *err describing it.
using ChunkSearch = std::function<int(int worker, uint64_t lo, uint64_t hi, uint64_t* hash, uint64_t* nonce,
                                      std::string* err)>;

// mh_search_multi with chunk > 0: one miner per worker, fed by the server's scheduler (sched.hpp)
// with chunks of exactly `chunk` nonces, one host thread each; a worker that fails hands its chunk
// back to the others, and so do workers whose thread could not start.  MH_OK with the minimum, or
// the first failure's code and text when no worker was left.
int search_chunks(int ndev, const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper, uint64_t chunk,
                  const ChunkSearch& search, uint64_t* out_hash, uint64_t* out_nonce, std::string* err,
                  const ThreadStart& start = {});

}  // namespace mh
