// tsan_multi.cpp -- mh_search_multi's shard coordinator (bitcoin-miner_amd/csrc/multi.cpp) driven
// with a stand-in search from up to 8 worker threads, built with -fsanitize=thread by
// tests/test_host_sanitize.py.  The GPU search is replaced by a recorder: each span it is handed
// "finds" a deterministic (hash, nonce) of the span, sleeps a little, and some workers fail
// (any of them, possibly all).  Invariants, for random ranges (up to 2^64 - 1, long enough for the
// dynamic tail) and random device lists (repeats allowed):
//   * success <=> at least one worker survived;
//   * the successful spans tile [lower, upper] exactly once (a failed worker's span is handed back
//     and searched by the others);
//   * the result is the lexicographic minimum over the successful spans;
//   * a failure returns the failing search's code and text;
//   * rates are recorded for the devices whose searches of >= 2^30 nonces succeeded;
// and, first, that a device listed k times gets 1/k of its rate per entry (repeated_devices).
//
//   tsan_multi <seed> <iterations>     exit 0 = every invariant held
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <atomic>
#include <chrono>
#include <functional>
#include <memory>
#include <mutex>
#include <random>
#include <set>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "../../bitcoin-miner_amd/csrc/multi.hpp"
#include "../../include/minehip.h"

namespace mh {
int set_error(int code, const char*) { return code; }  // the scheduler's error slot (minehip.cpp's is per thread)
}  // namespace mh

static int g_fail = 0;
#define CHECK(c)                                                                  \
    do {                                                                          \
        if (!(c)) {                                                               \
            fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                             \
            return;                                                               \
        }                                                                         \
    } while (0)

static uint64_t splitmix(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

struct Rec {
    uint64_t lo, hi, h, n;
};

static void one_case(std::mt19937_64& rng, int it) {
    const int ndev = 1 + (int)(rng() % 8);
    std::vector<int> devs((size_t)ndev);
    for (auto& d : devs) d = (int)(rng() % 4);
    std::vector<bool> fails((size_t)ndev, false);
    const int mode = (int)(rng() % 4);  // 0: none fail, 1: one, 2: random set, 3: all
    for (int i = 0; i < ndev; ++i)
        fails[(size_t)i] = mode == 3 || (mode == 1 && i == (int)(rng() % ndev)) || (mode == 2 && rng() % 3 == 0);
    uint64_t lower, upper;
    switch (rng() % 4) {
        case 0: lower = rng() % 100000; upper = lower + rng() % 50000; break;
        case 1: lower = rng() % (1ull << 40); upper = lower + (rng() % 3 + 1) * ((uint64_t)ndev << 35); break;
        case 2: lower = ~0ull - (rng() % (1ull << 44)); upper = ~0ull; break;
        default: lower = 0; upper = ~0ull; break;
    }
    const std::string msg = (it % 2) ? "cmu440" : std::string(60, 'x');
    mh::Prefix pre;
    mh::absorb_prefix((const uint8_t*)msg.data(), msg.size(), &pre);
    std::mutex mu;
    std::vector<Rec> done;
    std::atomic<int> calls{0};
    const mh::SpanSearch search = [&](int worker, int dev, uint64_t lo, uint64_t hi, uint64_t* h, uint64_t* n,
                                      uint64_t* ns, std::string* err) -> int {
        (void)dev;
        calls++;
        std::this_thread::sleep_for(std::chrono::microseconds(splitmix(lo ^ (uint64_t)worker) % 300));
        if (fails[(size_t)worker]) {
            *err = "stand-in failure of worker " + std::to_string(worker);
            return MH_EHIP;
        }
        *h = splitmix(lo * 31 + hi);
        *n = lo + splitmix(hi) % (hi - lo + 1 == 0 ? 1 : hi - lo + 1);
        *ns = 1 + (hi - lo) / 50;  // ~50 nonces per ns
        std::lock_guard<std::mutex> lk(mu);
        done.push_back(Rec{lo, hi, *h, *n});
        return MH_OK;
    };
    mh::PlanOpts opt;
    uint64_t oh = 0, on = 0;
    std::string err;
    const int rc = mh::search_shards(devs.data(), ndev, pre, lower, upper, opt, search, &oh, &on, &err);
    const bool survivor = std::count(fails.begin(), fails.end(), false) > 0;
    if (!survivor) {
        CHECK(rc == MH_EHIP);
        CHECK(err.find("stand-in failure") == 0);
        return;
    }
    CHECK(rc == MH_OK);
    std::sort(done.begin(), done.end(), [](const Rec& a, const Rec& b) { return a.lo < b.lo; });
    CHECK(!done.empty() && done.front().lo == lower && done.back().hi == upper);
    for (size_t k = 1; k < done.size(); ++k) CHECK(done[k - 1].hi + 1 == done[k].lo);
    uint64_t bh = ~0ull, bn = ~0ull;
    for (const auto& r : done)
        if (r.h < bh || (r.h == bh && r.n < bn)) {
            bh = r.h;
            bn = r.n;
        }
    CHECK(oh == bh && on == bn);
    for (const auto& r : done)
        if (r.hi - r.lo >= mh::kRateMinNonces - 1u) {
            // some device searched this span and recorded a rate (which one is not recorded here)
            bool any = false;
            for (int d : devs) any = any || mh::device_rate(d) > 0.0;
            CHECK(any);
            break;
        }
}

// A starter whose threads after the first k fail to start (as std::thread does when the process
// is out of threads): MINEHIP_TEST_SPAWN_LIMIT's stand-in.
static mh::ThreadStart limited(int k) {
    auto n = std::make_shared<std::atomic<int>>(0);
    return [n, k](std::function<void()> fn) {
        if ((*n)++ >= k) throw std::system_error(std::make_error_code(std::errc::resource_unavailable_try_again));
        return std::thread(std::move(fn));
    };
}

// Both coordinators (rate-weighted shards, fixed scheduler chunks) with only k of ndev host threads
// started: with k > 0 the started workers take the others' work and the job ends with the minimum
// over spans that tile the range once; with k = 0 the call fails with MH_EINTERNAL.
static void spawn_failures(std::mt19937_64& rng) {
    for (int ndev : {1, 2, 5, 8}) {
        for (int k : {0, 1, ndev - 1, ndev}) {
            if (k < 0 || (k == ndev - 1 && ndev == 1)) continue;
            for (int path = 0; path < 2; ++path) {
                const uint64_t lower = rng() % (1ull << 40);
                const uint64_t upper = lower + (rng() % 4 + 1) * ((uint64_t)ndev << 34);
                std::mutex mu;
                std::vector<Rec> done;
                std::set<int> workers;
                auto rec = [&](int worker, uint64_t lo, uint64_t hi, uint64_t* h, uint64_t* n) {
                    std::this_thread::sleep_for(std::chrono::microseconds(splitmix(lo) % 200));
                    *h = splitmix(lo * 31 + hi);
                    *n = lo + splitmix(hi) % (hi - lo + 1);
                    std::lock_guard<std::mutex> lk(mu);
                    done.push_back(Rec{lo, hi, *h, *n});
                    workers.insert(worker);
                };
                std::vector<int> devs((size_t)ndev, 20);  // device 20: a rate of its own, unused elsewhere
                uint64_t oh = 0, on = 0;
                std::string err;
                int rc;
                if (path == 0) {
                    mh::Prefix pre;
                    mh::absorb_prefix((const uint8_t*)"cmu440", 6, &pre);
                    const mh::SpanSearch s = [&](int w, int, uint64_t lo, uint64_t hi, uint64_t* h, uint64_t* n,
                                                 uint64_t* ns, std::string*) {
                        rec(w, lo, hi, h, n);
                        *ns = 1 + (hi - lo) / 50;
                        return MH_OK;
                    };
                    rc = mh::search_shards(devs.data(), ndev, pre, lower, upper, mh::PlanOpts(), s, &oh, &on, &err,
                                           limited(k));
                } else {
                    const mh::ChunkSearch s = [&](int w, uint64_t lo, uint64_t hi, uint64_t* h, uint64_t* n,
                                                  std::string*) {
                        rec(w, lo, hi, h, n);
                        return MH_OK;
                    };
                    const uint64_t chunk = (upper - lower) / 40 + 1;
                    rc = mh::search_chunks(ndev, (const uint8_t*)"cmu440", 6, lower, upper, chunk, s, &oh, &on, &err,
                                           limited(k));
                }
                if (k == 0) {
                    CHECK(rc == MH_EINTERNAL && err.find("could not start") != std::string::npos && done.empty());
                    continue;
                }
                CHECK(rc == MH_OK);
                CHECK(*workers.rbegin() < k);  // only started workers searched
                std::sort(done.begin(), done.end(), [](const Rec& a, const Rec& b) { return a.lo < b.lo; });
                CHECK(!done.empty() && done.front().lo == lower && done.back().hi == upper);
                for (size_t i = 1; i < done.size(); ++i) CHECK(done[i - 1].hi + 1 == done[i].lo);
                uint64_t bh = ~0ull, bn = ~0ull;
                for (const auto& r : done)
                    if (r.h < bh || (r.h == bh && r.n < bn)) {
                        bh = r.h;
                        bn = r.n;
                    }
                CHECK(oh == bh && on == bn);
            }
        }
    }
}

// A device listed k times runs its k shards one after another, so each of its entries weighs 1/k of
// its rate and every physical device carries a share of the range in proportion to its own rate
// (devices 10..12: never listed by one_case, so their rates are only these).
static void repeated_devices() {
    mh::record_rate(10, 3.0e9, 1000000000ull);  // 3 slots per ns
    mh::record_rate(11, 3.0e9, 1000000000ull);
    mh::record_rate(12, 1.5e9, 1000000000ull);  // half as fast
    const int devs[5] = {10, 11, 10, 12, 10};
    const std::vector<double> w = mh::worker_weights(devs, 5);
    CHECK(w.size() == 5);
    CHECK(std::abs(w[0] - 1.0) < 1e-9 && std::abs(w[2] - 1.0) < 1e-9 && std::abs(w[4] - 1.0) < 1e-9);
    CHECK(std::abs(w[1] - 3.0) < 1e-9 && std::abs(w[3] - 1.5) < 1e-9);
    mh::Prefix pre;
    mh::absorb_prefix((const uint8_t*)"cmu440", 6, &pre);
    mh::MultiPlan mp;
    mh::multi_plan(pre, 1ull << 39, (1ull << 39) + (1ull << 34), mh::PlanOpts(), w, &mp);  // no dynamic tail
    CHECK(mp.tail.empty());
    double cost[3] = {0, 0, 0};
    for (int i = 0; i < 5; ++i)
        if (!mp.head[(size_t)i].empty)
            cost[devs[i] - 10] += mh::segments_cost(mp.segs, mp.head[(size_t)i].lo, mp.head[(size_t)i].hi);
    CHECK(std::abs(cost[0] / cost[1] - 1.0) < 1e-6 && std::abs(cost[2] / cost[1] - 0.5) < 1e-6);
}

int main(int argc, char** argv) {
    const uint64_t seed = argc > 1 ? strtoull(argv[1], nullptr, 10) : 440;
    const int iters = argc > 2 ? atoi(argv[2]) : 100;
    std::mt19937_64 rng(seed);
    repeated_devices();
    spawn_failures(rng);
    for (int it = 0; it < iters; ++it) one_case(rng, it);
    printf("iterations=%d failures=%d\n", iters, g_fail);
    return g_fail ? 1 : 0;
}
