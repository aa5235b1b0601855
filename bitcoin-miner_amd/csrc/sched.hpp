// sched.hpp -- the bitcoin server's chunk scheduler (SURVEY.md §8(f) N2;
// reference stub bitcoin/server/server.go:62).  Host-only C++, no HIP: used by
// the mh_sched_* / mh_server_* C-ABI (include/minehip_server.h) and by
// mh_search_multi, whose per-device worker threads are its miners.
//
// A job is a client's Request range [lower, upper] (message.go:27-34).  It is
// cut into chunks on demand, one outstanding chunk per miner, sized from the
// miner's measured rate and the work left (guided self-scheduling), and
// merged by the lexicographic min of (hash, nonce) -- associative and
// commutative, so the answer does not depend on chunking, order or
// reassignment (tests/test_sched.py checks exactly that against the oracle).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/minehip_server.h"

namespace mh {

class Scheduler {
  public:
    // opts must be valid (see valid_opts)
    explicit Scheduler(const mh_sched_opts& opts);

    static bool valid_opts(const mh_sched_opts& o);

    int add_miner(int64_t id);
    int remove_miner(int64_t id);
    int64_t submit(int64_t client, const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper);
    int drop_client(int64_t client);
    int next(int64_t miner, uint64_t now_ns, mh_assignment* out);
    int job_msg(int64_t job, std::string* out);
    int result(int64_t miner, uint64_t hash, uint64_t nonce, uint64_t now_ns, mh_completion* out);
    void stats(mh_sched_stats* out);
    // true when no live job is left (all done or cancelled and drained)
    bool idle_jobs();

  private:
    using u128 = unsigned __int128;
    struct Job {
        int64_t id, client;
        std::string msg;
        uint64_t lower, upper;
        uint64_t next;       // first nonce never handed out
        bool exhausted;      // every nonce handed out at least once
        std::deque<std::pair<uint64_t, uint64_t>> requeue;  // chunks of lost miners
        uint64_t outstanding;
        uint64_t best_hash, best_nonce;
        bool cancelled;
        u128 pending() const;  // nonces not handed out (fresh + requeued)
    };
    struct Miner {
        int64_t id;
        bool busy;
        int64_t job;
        uint64_t lo, hi, t0;
        double rate;  // nonces per ns, EWMA; 0 before the first chunk
    };

    Job* find_job(int64_t id);
    Miner* find_miner(int64_t id);
    void erase_job(int64_t id);
    uint64_t chunk_size(const Miner& m, const Job& j) const;
    bool take(Job& j, uint64_t c, uint64_t* lo, uint64_t* hi);

    std::mutex mu_;
    mh_sched_opts o_;
    std::vector<std::unique_ptr<Job>> jobs_;  // submission order
    std::vector<Miner> miners_;               // join order
    size_t rr_ = 0;                           // round-robin cursor into jobs_
    int64_t next_job_ = 0;
    mh_sched_stats st_{};
};

}  // namespace mh
