// tsan_sched.cpp -- the server scheduler (bitcoin-miner_amd/csrc/sched.cpp,
// server loop csrc/server.cpp) driven from many threads at once, built with
// -fsanitize=thread by tests/test_host_sanitize.py.  The C-ABI says every
// mh_sched_* / mh_server_* call is thread-safe; this is the race check.
//
// Miner threads loop on mh_sched_next / mh_sched_result, "searching" each
// chunk with a cheap stand-in hash (splitmix64 of the nonce and the job's
// message: the scheduler never looks at hashes except to merge them).  One
// thread submits jobs, another drops a client and removes / re-adds miners.
// Every finished job's answer must equal the lexicographic min of the stand-in
// hash over its whole range, computed directly.
//
//   tsan_sched <seed>     exit 0 = every invariant held
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../bitcoin-miner_amd/csrc/sched.hpp"
#include "../../include/minehip.h"
#include "../../include/minehip_server.h"

namespace mh {
int set_error(int code, const char*) { return code; }
}  // namespace mh

static std::atomic<int> g_fail{0};
#define CHECK(c)                                                                  \
    do {                                                                          \
        if (!(c)) {                                                               \
            fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
            g_fail++;                                                             \
        }                                                                         \
    } while (0)

static uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
static uint64_t fake_hash(uint64_t key, uint64_t n) { return mix(key ^ mix(n)) >> 8; }  // ties possible
static uint64_t msg_key(const std::string& m) {
    uint64_t k = 1469598103934665603ull;
    for (unsigned char c : m) k = (k ^ c) * 1099511628211ull;
    return k;
}
static void scan(uint64_t key, uint64_t lo, uint64_t hi, uint64_t* h, uint64_t* n) {
    *h = ~0ull;
    *n = ~0ull;
    for (uint64_t x = lo;; ++x) {
        const uint64_t v = fake_hash(key, x);
        if (v < *h) {  // strict <: the lowest nonce keeps a tie
            *h = v;
            *n = x;
        }
        if (x == hi) break;
    }
}

int main(int argc, char** argv) {
    const uint64_t seed = argc > 1 ? strtoull(argv[1], nullptr, 10) : 440;
    mh_sched_opts o;
    mh_sched_default_opts(&o);
    o.init_chunk = 257;
    o.min_chunk = 31;
    o.max_chunk = 4096;
    o.target_ns = 20000;
    mh_sched* s = mh_sched_create(&o);
    CHECK(s != nullptr);
    const int kMiners = 6, kJobs = 80;
    for (int m = 0; m < kMiners; ++m) CHECK(mh_sched_add_miner(s, m) == MH_OK);

    std::mutex mu;
    std::map<int64_t, std::pair<uint64_t, uint64_t>> want;  // job -> expected (hash, nonce)
    std::map<int64_t, int64_t> client_of;
    std::map<int64_t, std::pair<uint64_t, uint64_t>> got;
    std::atomic<int> submitted{0};
    std::atomic<bool> stop{false};
    auto now = [] {
        return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                   std::chrono::steady_clock::now().time_since_epoch())
            .count();
    };

    std::thread submitter([&] {
        std::mt19937_64 r(seed);
        for (int j = 0; j < kJobs; ++j) {
            std::string m = "job" + std::to_string(j) + std::string(r() % 70, 'x');
            const uint64_t lo = (j % 5 == 0) ? ~0ull - (r() % 3000) : r() % 1000000;
            const uint64_t hi = (j % 5 == 0) ? ~0ull : lo + r() % 100000;
            uint64_t h, n;
            scan(msg_key(m), lo, hi, &h, &n);
            const int64_t client = 1000 + j;
            std::lock_guard<std::mutex> lk(mu);  // job id and expectation recorded together
            const int64_t id = mh_sched_submit(s, client, (const uint8_t*)m.data(), m.size(), lo, hi);
            CHECK(id >= 0);
            want[id] = {h, n};
            client_of[id] = client;
            submitted++;
        }
    });

    std::vector<std::thread> miners;
    for (int m = 0; m < kMiners; ++m) {
        miners.emplace_back([&, m] {
            std::string buf(2048, '\0');
            while (!stop) {
                mh_assignment a;
                if (mh_sched_next(s, m, now(), &a) != 1) {
                    std::this_thread::yield();
                    continue;
                }
                size_t len = 0;
                // a job stays alive while one of its chunks is out, cancelled or not
                const int jr = mh_sched_job_msg(s, a.job, (uint8_t*)&buf[0], buf.size(), &len);
                CHECK(jr == MH_OK);
                if (jr != MH_OK) {  // requeue the chunk rather than report an unscanned one
                    mh_sched_remove_miner(s, m);
                    mh_sched_add_miner(s, m);
                    continue;
                }
                uint64_t h, n;
                scan(msg_key(std::string(buf.data(), len)), a.lower, a.upper, &h, &n);
                mh_completion c;
                const int r = mh_sched_result(s, m, h, n, now(), &c);
                CHECK(r == 0 || r == 1);
                if (r == 1) {
                    std::lock_guard<std::mutex> lk(mu);
                    CHECK(!got.count(c.job));
                    got[c.job] = {c.hash, c.nonce};
                    CHECK(client_of.count(c.job) && client_of[c.job] == c.client);
                }
            }
        });
    }

    // churn: a miner leaves mid-chunk and comes back; one client is dropped
    std::thread churn([&] {
        std::mt19937_64 r(seed + 1);
        for (int k = 0; k < 50 && !stop; ++k) {
            std::this_thread::sleep_for(std::chrono::microseconds(200 + r() % 500));
            const int64_t extra = 100 + k;
            CHECK(mh_sched_add_miner(s, extra) == MH_OK);
            mh_assignment a;
            (void)mh_sched_next(s, extra, now(), &a);
            CHECK(mh_sched_remove_miner(s, extra) == MH_OK);  // its chunk goes back
        }
        while (submitted < 3) std::this_thread::yield();
        mh_sched_drop_client(s, 1000 + 2);  // job 2's client is gone
    });

    submitter.join();
    churn.join();
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::seconds(120);
    for (;;) {
        mh_sched_stats st;
        mh_sched_stats_read(s, &st);
        if (st.jobs == 0) break;
        if (std::chrono::steady_clock::now() > t_end) {
            CHECK(!"jobs left after 120 s");
            break;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
    stop = true;
    for (auto& t : miners) t.join();

    int checked = 0;
    for (auto& kv : want) {
        auto it = got.find(kv.first);
        if (client_of[kv.first] == 1000 + 2 && it == got.end()) continue;  // cancelled
        CHECK(it != got.end());
        if (it != got.end()) {
            CHECK(it->second == kv.second);
            ++checked;
        }
    }
    CHECK(checked >= kJobs - 1);
    mh_sched_destroy(s);
    printf("jobs_checked=%d failures=%d\n", checked, g_fail.load());
    return g_fail ? 1 : 0;
}
