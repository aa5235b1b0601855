// sched.cpp -- Scheduler (sched.hpp) and the mh_sched_* C-ABI
// (include/minehip_server.h).  SURVEY.md §8(f) N2; reference stub
// bitcoin/server/server.go:62.
#include "sched.hpp"

#include <string.h>

#include <algorithm>

#include "../../include/minehip.h"

namespace mh {
int set_error(int code, const char* what);

namespace {
inline bool lex_less(uint64_t ha, uint64_t na, uint64_t hb, uint64_t nb) {
    return ha < hb || (ha == hb && na < nb);
}
}  // namespace

bool Scheduler::valid_opts(const mh_sched_opts& o) {
    return o.init_chunk >= 1 && o.min_chunk >= 1 && o.max_chunk >= o.min_chunk && o.target_ns >= 1;
}

Scheduler::Scheduler(const mh_sched_opts& opts) : o_(opts) {}

Scheduler::u128 Scheduler::Job::pending() const {
    u128 p = exhausted ? 0 : (u128)(upper - next) + 1u;
    for (const auto& r : requeue) p += (u128)(r.second - r.first) + 1u;
    return p;
}

Scheduler::Job* Scheduler::find_job(int64_t id) {
    for (auto& j : jobs_)
        if (j->id == id) return j.get();
    return nullptr;
}

Scheduler::Miner* Scheduler::find_miner(int64_t id) {
    for (auto& m : miners_)
        if (m.id == id) return &m;
    return nullptr;
}

void Scheduler::erase_job(int64_t id) {
    for (size_t i = 0; i < jobs_.size(); ++i) {
        if (jobs_[i]->id != id) continue;
        jobs_.erase(jobs_.begin() + (ptrdiff_t)i);
        if (rr_ > i) --rr_;
        if (rr_ >= jobs_.size()) rr_ = 0;
        return;
    }
}

// rate x target, capped at the job's fair share of what is left (guided
// self-scheduling: half of an even split, so the tail is spread over every
// miner; a lone miner has no tail to share), clamped.
uint64_t Scheduler::chunk_size(const Miner& m, const Job& j) const {
    double want = m.rate > 0.0 ? m.rate * (double)o_.target_ns : (double)o_.init_chunk;
    const size_t nm = miners_.size();
    const u128 share = j.pending() / (u128)(nm > 1 ? 2u * nm : 1u);
    if ((double)share < want) want = (double)share;
    if (want < (double)o_.min_chunk) want = (double)o_.min_chunk;
    if (want > (double)o_.max_chunk) want = (double)o_.max_chunk;
    const uint64_t c = (uint64_t)want;
    return c < 1 ? 1 : c;
}

// Cut up to c nonces from the job: requeued chunks first (oldest loss first).
bool Scheduler::take(Job& j, uint64_t c, uint64_t* lo, uint64_t* hi) {
    if (!j.requeue.empty()) {
        auto& r = j.requeue.front();
        *lo = r.first;
        if (r.second - r.first <= c - 1u) {
            *hi = r.second;
            j.requeue.pop_front();
        } else {
            *hi = r.first + (c - 1u);
            r.first = *hi + 1u;
        }
        return true;
    }
    if (j.exhausted) return false;
    *lo = j.next;
    if (j.upper - j.next <= c - 1u) {
        *hi = j.upper;
        j.exhausted = true;
    } else {
        *hi = j.next + (c - 1u);
        j.next = *hi + 1u;
    }
    return true;
}

int Scheduler::add_miner(int64_t id) {
    std::lock_guard<std::mutex> lk(mu_);
    if (find_miner(id)) return set_error(MH_EINVAL, "miner already joined");
    miners_.push_back(Miner{id, false, -1, 0, 0, 0, 0.0});
    return MH_OK;
}

int Scheduler::remove_miner(int64_t id) {
    std::lock_guard<std::mutex> lk(mu_);
    for (size_t i = 0; i < miners_.size(); ++i) {
        Miner& m = miners_[i];
        if (m.id != id) continue;
        if (m.busy) {
            if (Job* j = find_job(m.job)) {
                j->outstanding -= 1u;
                if (!j->cancelled) {
                    j->requeue.emplace_front(m.lo, m.hi);
                    st_.chunks_requeued += 1u;
                } else if (j->outstanding == 0) {
                    erase_job(j->id);
                }
            }
        }
        miners_.erase(miners_.begin() + (ptrdiff_t)i);
        return MH_OK;
    }
    return set_error(MH_EINVAL, "unknown miner");
}

int64_t Scheduler::submit(int64_t client, const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper) {
    if (!msg && len) return set_error(MH_EINVAL, "msg is NULL");
    if (len > MH_MAX_MSG_LEN) return set_error(MH_ETOOLONG, "message longer than MH_MAX_MSG_LEN");
    if (lower > upper) return set_error(MH_ERANGE, "lower > upper");
    std::lock_guard<std::mutex> lk(mu_);
    std::unique_ptr<Job> j(new Job());
    j->id = next_job_++;
    j->client = client;
    j->msg.assign((const char*)msg, len);
    j->lower = lower;
    j->upper = upper;
    j->next = lower;
    j->exhausted = false;
    j->outstanding = 0;
    j->best_hash = j->best_nonce = ~0ull;
    j->cancelled = false;
    jobs_.push_back(std::move(j));
    return jobs_.back()->id;
}

int Scheduler::drop_client(int64_t client) {
    std::lock_guard<std::mutex> lk(mu_);
    int n = 0;
    std::vector<int64_t> gone;
    for (auto& j : jobs_) {
        if (j->client != client || j->cancelled) continue;
        j->cancelled = true;
        j->exhausted = true;
        j->requeue.clear();
        st_.jobs_cancelled += 1u;
        ++n;
        if (j->outstanding == 0) gone.push_back(j->id);
    }
    for (int64_t id : gone) erase_job(id);
    return n;
}

int Scheduler::next(int64_t miner, uint64_t now_ns, mh_assignment* out) {
    if (!out) return set_error(MH_EINVAL, "NULL output");
    std::lock_guard<std::mutex> lk(mu_);
    Miner* m = nullptr;
    if (miner >= 0) {
        m = find_miner(miner);
        if (!m) return set_error(MH_EINVAL, "unknown miner");
        if (m->busy) return 0;
    } else {
        for (auto& x : miners_)
            if (!x.busy) {
                m = &x;
                break;
            }
        if (!m) return 0;
    }
    const size_t nj = jobs_.size();
    for (size_t k = 0; k < nj; ++k) {
        const size_t idx = (rr_ + k) % nj;
        Job& j = *jobs_[idx];
        if (j.cancelled) continue;
        uint64_t lo, hi;
        if (!take(j, chunk_size(*m, j), &lo, &hi)) continue;
        rr_ = (idx + 1) % nj;
        j.outstanding += 1u;
        m->busy = true;
        m->job = j.id;
        m->lo = lo;
        m->hi = hi;
        m->t0 = now_ns;
        st_.chunks_assigned += 1u;
        out->miner = m->id;
        out->job = j.id;
        out->lower = lo;
        out->upper = hi;
        out->msg_len = j.msg.size();
        return 1;
    }
    return 0;
}

int Scheduler::job_msg(int64_t job, std::string* out) {
    std::lock_guard<std::mutex> lk(mu_);
    Job* j = find_job(job);
    if (!j) return set_error(MH_EINVAL, "unknown job");
    *out = j->msg;
    return MH_OK;
}

int Scheduler::result(int64_t miner, uint64_t hash, uint64_t nonce, uint64_t now_ns, mh_completion* out) {
    std::lock_guard<std::mutex> lk(mu_);
    Miner* m = find_miner(miner);
    if (!m || !m->busy) return set_error(MH_EINVAL, "Result from a miner with no chunk out");
    m->busy = false;
    Job* j = find_job(m->job);
    if (!j) return 0;  // cannot happen: a job lives while chunks are out
    if (nonce < m->lo || nonce > m->hi) {
        j->outstanding -= 1u;
        if (!j->cancelled) {
            j->requeue.emplace_front(m->lo, m->hi);
            st_.chunks_requeued += 1u;
        } else if (j->outstanding == 0) {
            erase_job(j->id);
        }
        return set_error(MH_ERANGE, "Result nonce outside the miner's chunk");
    }
    const double cnt = (double)(m->hi - m->lo) + 1.0;
    if (now_ns > m->t0) {
        const double r = cnt / (double)(now_ns - m->t0);
        m->rate = m->rate > 0.0 ? 0.5 * m->rate + 0.5 * r : r;
    }
    st_.chunks_done += 1u;
    st_.nonces_done += m->hi - m->lo + 1u;  // wraps only for a single 2^64 chunk
    j->outstanding -= 1u;
    if (!j->cancelled && lex_less(hash, nonce, j->best_hash, j->best_nonce)) {
        j->best_hash = hash;
        j->best_nonce = nonce;
    }
    if (j->outstanding != 0 || (!j->cancelled && (!j->exhausted || !j->requeue.empty()))) return 0;
    if (j->cancelled) {
        erase_job(j->id);
        return 0;
    }
    if (out) {
        out->job = j->id;
        out->client = j->client;
        out->hash = j->best_hash;
        out->nonce = j->best_nonce;
    }
    st_.jobs_done += 1u;
    erase_job(j->id);
    return 1;
}

void Scheduler::stats(mh_sched_stats* out) {
    std::lock_guard<std::mutex> lk(mu_);
    *out = st_;
    out->miners = miners_.size();
    out->idle_miners = 0;
    for (const auto& m : miners_) out->idle_miners += m.busy ? 0u : 1u;
    out->jobs = jobs_.size();
}

bool Scheduler::idle_jobs() {
    std::lock_guard<std::mutex> lk(mu_);
    return jobs_.empty();
}

}  // namespace mh

struct mh_sched {
    mh::Scheduler s;
    explicit mh_sched(const mh_sched_opts& o) : s(o) {}
};

extern "C" {

void mh_sched_default_opts(mh_sched_opts* o) {
    if (!o) return;
    o->init_chunk = 1ull << 30;
    o->min_chunk = 1ull << 24;
    o->max_chunk = 1ull << 38;
    o->target_ns = 250000000ull;
}

mh_sched* mh_sched_create(const mh_sched_opts* opts) {
    mh_sched_opts o;
    mh_sched_default_opts(&o);
    if (opts) o = *opts;
    if (!mh::Scheduler::valid_opts(o)) {
        mh::set_error(MH_EINVAL, "bad scheduler options");
        return nullptr;
    }
    return new mh_sched(o);
}

void mh_sched_destroy(mh_sched* s) { delete s; }

#define MH_NEED(s) \
    if (!(s)) return mh::set_error(MH_EINVAL, "NULL scheduler")

int mh_sched_add_miner(mh_sched* s, int64_t miner) {
    MH_NEED(s);
    return s->s.add_miner(miner);
}

int mh_sched_remove_miner(mh_sched* s, int64_t miner) {
    MH_NEED(s);
    return s->s.remove_miner(miner);
}

int64_t mh_sched_submit(mh_sched* s, int64_t client, const uint8_t* msg, size_t len, uint64_t lower,
                        uint64_t upper) {
    MH_NEED(s);
    return s->s.submit(client, msg, len, lower, upper);
}

int mh_sched_drop_client(mh_sched* s, int64_t client) {
    MH_NEED(s);
    return s->s.drop_client(client);
}

int mh_sched_next(mh_sched* s, int64_t miner, uint64_t now_ns, mh_assignment* out) {
    MH_NEED(s);
    return s->s.next(miner, now_ns, out);
}

int mh_sched_job_msg(mh_sched* s, int64_t job, uint8_t* buf, size_t cap, size_t* len) {
    MH_NEED(s);
    std::string m;
    int rc = s->s.job_msg(job, &m);
    if (rc) return rc;
    if (len) *len = m.size();
    if (m.size() > cap || (!buf && !m.empty())) return mh::set_error(MH_ETOOLONG, "buffer too small");
    if (!m.empty()) memcpy(buf, m.data(), m.size());
    return MH_OK;
}

int mh_sched_result(mh_sched* s, int64_t miner, uint64_t hash, uint64_t nonce, uint64_t now_ns,
                    mh_completion* out) {
    MH_NEED(s);
    return s->s.result(miner, hash, nonce, now_ns, out);
}

int mh_sched_stats_read(mh_sched* s, mh_sched_stats* out) {
    MH_NEED(s);
    if (!out) return mh::set_error(MH_EINVAL, "NULL output");
    s->s.stats(out);
    return MH_OK;
}

}  // extern "C"
