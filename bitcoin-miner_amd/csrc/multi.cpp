// multi.cpp -- see multi.hpp.
#include "multi.hpp"

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>

#include "../../include/minehip.h"
#include "sched.hpp"

namespace mh {
namespace {

std::mutex g_rate_mu;
std::vector<double> g_rate;  // per device: slots per ns (EWMA over its searches), 0 = not measured

// The span split into `parts` contiguous near-equal pieces (a failed worker's span, handed back).
std::vector<Span> split_even(const Span& s, int parts) {
    std::vector<Span> out;
    const unsigned __int128 n = (unsigned __int128)(s.hi - s.lo) + 1u;
    unsigned __int128 prev = 0;
    for (int k = 1; k <= parts; ++k) {
        const unsigned __int128 pos = n * (unsigned)k / (unsigned)parts;
        if (pos > prev) out.push_back(Span{(uint64_t)(s.lo + prev), (uint64_t)(s.lo + (pos - 1u)), false});
        prev = pos;
    }
    return out;
}

std::thread start_thread(const ThreadStart& start, std::function<void()> fn) {
    return start ? start(std::move(fn)) : std::thread(std::move(fn));
}

}  // namespace

std::vector<double> worker_weights(const int* devs, int ndev) {
    std::lock_guard<std::mutex> lk(g_rate_mu);
    std::vector<double> w((size_t)ndev, 0.0);
    double sum = 0.0;
    int known = 0;
    for (int i = 0; i < ndev; ++i) {
        const double r = (devs[i] >= 0 && (size_t)devs[i] < g_rate.size()) ? g_rate[(size_t)devs[i]] : 0.0;
        w[(size_t)i] = r;
        if (r > 0.0) {
            sum += r;
            ++known;
        }
    }
    const double fill = known ? sum / known : 1.0;
    for (auto& x : w)
        if (x <= 0.0) x = fill;
    // A device listed k times runs its k shards one after another (one search at a time per
    // device), so each entry gets 1/k of its device's rate: every physical device then carries a
    // share of the range in proportion to its own rate.
    for (int i = 0; i < ndev; ++i) {
        int k = 0;
        for (int j = 0; j < ndev; ++j) k += devs[j] == devs[i];
        w[(size_t)i] /= (double)k;
    }
    return w;
}

void record_rate(int dev, double slots, uint64_t ns) {
    if (dev < 0 || ns == 0 || slots <= 0.0) return;
    std::lock_guard<std::mutex> lk(g_rate_mu);
    if ((size_t)dev >= g_rate.size()) g_rate.resize((size_t)dev + 1, 0.0);
    const double r = slots / (double)ns;
    g_rate[(size_t)dev] = g_rate[(size_t)dev] > 0.0 ? 0.5 * g_rate[(size_t)dev] + 0.5 * r : r;
}

double device_rate(int dev) {
    std::lock_guard<std::mutex> lk(g_rate_mu);
    return (dev >= 0 && (size_t)dev < g_rate.size()) ? g_rate[(size_t)dev] : 0.0;
}

void multi_plan(const Prefix& pre, uint64_t lower, uint64_t upper, const PlanOpts& opt,
                const std::vector<double>& w, MultiPlan* mp) {
    cost_segments(pre, lower, upper, opt, &mp->segs);
    const size_t n = w.size();
    const unsigned __int128 total = (unsigned __int128)(upper - lower) + 1u;
    const size_t T = (n > 1 && total / n >= kTailMinPerWorker) ? 2 * n : 0;
    std::vector<double> ww = w;
    double wsum = 0.0;
    for (double x : w) wsum += x;
    for (size_t k = 0; k < T; ++k) ww.push_back(wsum / (double)(kTailDiv - 1) / (double)T);  // tail = 1/16
    std::vector<Span> all;
    split_by_cost(mp->segs, ww, &all);
    mp->head.assign(all.begin(), all.begin() + (ptrdiff_t)n);
    mp->tail.clear();
    for (size_t k = n; k < all.size(); ++k)
        if (!all[k].empty) mp->tail.push_back(all[k]);
}

int search_shards(const int* devs, int ndev, const Prefix& pre, uint64_t lower, uint64_t upper,
                  const PlanOpts& opt, const SpanSearch& search, uint64_t* out_hash, uint64_t* out_nonce,
                  std::string* err, const ThreadStart& start) {
    MultiPlan mp;
    multi_plan(pre, lower, upper, opt, worker_weights(devs, ndev), &mp);
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Span> queue(mp.tail.begin(), mp.tail.end());
    int outstanding = 0, alive = ndev, first_err = 0;
    for (const auto& s : mp.head) outstanding += s.empty ? 0 : 1;
    std::string err_msg;
    uint64_t bh = ~0ull, bn = ~0ull;
    bool any = false;
    auto worker = [&](int i) {
        Span cur = mp.head[(size_t)i];
        bool have = !cur.empty;
        for (;;) {
            if (have) {
                uint64_t h = 0, nn = 0, ns = 0;
                std::string e;
                const int r = search(i, devs[i], cur.lo, cur.hi, &h, &nn, &ns, &e);
                // a device's rate comes from long spans of steady buckets only: a shard holding the
                // small buckets of a range would otherwise read as a slower device (multi.hpp)
                if (r == MH_OK && cur.hi - cur.lo >= kRateMinNonces - 1u &&
                    unsteady_share(mp.segs, cur.lo, cur.hi) < kRateMaxUnsteady)
                    record_rate(devs[i], segments_cost(mp.segs, cur.lo, cur.hi), ns);
                std::lock_guard<std::mutex> lk(mu);
                --outstanding;
                if (r != MH_OK) {
                    // hand the span back, cut for the workers still running, and leave
                    if (!first_err) {
                        first_err = r;
                        err_msg = e;
                    }
                    --alive;
                    const auto parts = split_even(cur, std::max(1, alive));
                    queue.insert(queue.begin(), parts.begin(), parts.end());
                    cv.notify_all();
                    return;
                }
                if (!any || h < bh || (h == bh && nn < bn)) {
                    bh = h;
                    bn = nn;
                    any = true;
                }
                cv.notify_all();
            }
            std::unique_lock<std::mutex> lk(mu);
            // wait for work: a tail chunk, or a span a failed worker handed back
            cv.wait(lk, [&] { return !queue.empty() || outstanding == 0; });
            if (queue.empty()) return;  // nothing queued and nothing running: done
            cur = queue.front();
            queue.pop_front();
            ++outstanding;
            have = true;
        }
    };
    std::vector<std::thread> th;
    try {
        for (int i = 0; i < ndev; ++i) th.push_back(start_thread(start, [&worker, i] { worker(i); }));
    } catch (...) {
        // out of threads: the workers that started take the heads of those that did not
        std::lock_guard<std::mutex> lk(mu);
        for (size_t i = th.size(); i < (size_t)ndev; ++i)
            if (!mp.head[i].empty) {
                queue.push_back(mp.head[i]);
                --outstanding;
            }
        alive -= ndev - (int)th.size();
        if (!first_err) {
            first_err = MH_EINTERNAL;
            err_msg = "could not start a host thread per device";
        }
        cv.notify_all();
    }
    for (auto& t : th) t.join();
    if (!queue.empty() || !any) {
        *err = err_msg.empty() ? "every device failed" : err_msg;
        return first_err ? first_err : MH_EHIP;
    }
    *out_hash = bh;
    *out_nonce = bn;
    return MH_OK;
}

int search_chunks(int ndev, const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper, uint64_t chunk,
                  const ChunkSearch& search, uint64_t* out_hash, uint64_t* out_nonce, std::string* err,
                  const ThreadStart& start) {
    mh_sched_opts o;
    mh_sched_default_opts(&o);
    o.init_chunk = o.min_chunk = o.max_chunk = chunk;
    Scheduler sched(o);
    for (int i = 0; i < ndev; ++i) sched.add_miner(i);
    if (sched.submit(0, msg, len, lower, upper) < 0) {
        *err = "internal: submit failed";
        return MH_EINTERNAL;
    }
    std::mutex mu;
    std::condition_variable cv;
    uint64_t gen = 0;  // bumped on every completion or worker loss
    int alive = ndev, first_err = 0;
    bool done = false;
    mh_completion res{};
    std::string err_msg;
    auto now = []() {
        return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
    };
    auto miner = [&](int i) {
        for (;;) {
            uint64_t seen;
            {
                std::lock_guard<std::mutex> lk(mu);
                if (done) return;
                seen = gen;
            }
            mh_assignment a;
            if (sched.next(i, now(), &a) != 1) {
                // nothing to hand out: wait for the job to finish, or for a failed worker's chunk
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return done || gen != seen; });
                continue;
            }
            uint64_t h = 0, nn = 0;
            std::string e;
            const int r = search(i, a.lower, a.upper, &h, &nn, &e);
            if (r) {
                sched.remove_miner(i);  // its chunk goes back to the job
                std::lock_guard<std::mutex> lk(mu);
                if (!first_err) {
                    first_err = r;
                    err_msg = e;
                }
                if (--alive == 0) done = true;
                ++gen;
                cv.notify_all();
                return;
            }
            mh_completion c;
            const int q = sched.result(i, h, nn, now(), &c);
            std::lock_guard<std::mutex> lk(mu);
            if (q == 1) {
                res = c;
                done = true;
            }
            ++gen;
            cv.notify_all();
        }
    };
    std::vector<std::thread> th;
    try {
        for (int i = 0; i < ndev; ++i) th.push_back(start_thread(start, [&miner, i] { miner(i); }));
    } catch (...) {
        // out of threads: the miners that did not start leave the scheduler (their chunks, if
        // any, go back to the job) and the started ones finish the job
        for (size_t i = th.size(); i < (size_t)ndev; ++i) sched.remove_miner((int64_t)i);
        std::lock_guard<std::mutex> lk(mu);
        alive -= ndev - (int)th.size();
        if (!first_err) {
            first_err = MH_EINTERNAL;
            err_msg = "could not start a host thread per device";
        }
        if (alive == 0) done = true;
        ++gen;
        cv.notify_all();
    }
    for (auto& t : th) t.join();
    if (alive == 0) {
        *err = err_msg.empty() ? "every device failed" : err_msg;
        return first_err ? first_err : MH_EHIP;
    }
    *out_hash = res.hash;
    *out_nonce = res.nonce;
    return MH_OK;
}

}  // namespace mh
