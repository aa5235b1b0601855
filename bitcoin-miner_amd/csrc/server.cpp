// server.cpp -- the bitcoin server's message loop (reference stub
// bitcoin/server/server.go:62) over the Scheduler, as the
// mh_server_* C-ABI (include/minehip_server.h).
//
// Transport-agnostic: the Go server keeps its lsp.Server (server.go:12-14)
// and, for every Read, calls mh_server_read (payload) or mh_server_lost
// (error), then drains mh_server_pop_write into lsp.Server.Write.  Payloads
// are Go encoding/json bitcoin.Messages (msgcodec.hpp):
//   Join (message.go:47)     -> the connection becomes a miner;
//   Request (message.go:27)  -> a job for the connection (a client);
//   Result (message.go:38)   -> the miner's chunk is done;
// and every idle miner is handed a chunk as a Request carrying the job's
// Data.  A finished job writes NewResult(hash, nonce) to its client.
#include <string.h>

#include <deque>
#include <set>
#include <string>
#include <utility>

#include "../../include/minehip.h"
#include "msgcodec.hpp"
#include "sched.hpp"

struct mh_server {
    std::mutex mu;  // serialises read/lost/pop (the scheduler locks itself too)
    mh::Scheduler s;
    std::set<int64_t> miners;
    std::deque<std::pair<int64_t, std::string>> out;
    explicit mh_server(const mh_sched_opts& o) : s(o) {}

    // hand every idle miner a chunk
    int dispatch(uint64_t now) {
        mh_assignment a;
        for (;;) {
            const int r = s.next(-1, now, &a);
            if (r < 0) return r;
            if (r == 0) return MH_OK;
            std::string m;
            const int rc = s.job_msg(a.job, &m);
            if (rc) return rc;
            out.emplace_back(a.miner, mh::encode(1, (const uint8_t*)m.data(), m.size(), a.lower, a.upper, 0, 0));
        }
    }
};

extern "C" {

mh_server* mh_server_create(const mh_sched_opts* opts) {
    mh_sched_opts o;
    mh_sched_default_opts(&o);
    if (opts) o = *opts;
    if (!mh::Scheduler::valid_opts(o)) {
        mh::set_error(MH_EINVAL, "bad scheduler options");
        return nullptr;
    }
    return new mh_server(o);
}

void mh_server_destroy(mh_server* v) { delete v; }

int mh_server_read(mh_server* v, int64_t conn, const char* payload, size_t len, uint64_t now_ns) {
    if (!v || (!payload && len)) return mh::set_error(MH_EINVAL, "bad arguments");
    std::lock_guard<std::mutex> lk(v->mu);
    mh::Msg m;
    if (!mh::decode(payload ? payload : "", len, &m))
        return mh::set_error(MH_EINVAL, "payload is not a JSON bitcoin.Message");
    int rc = MH_OK;
    switch (m.type) {
        case 0:  // Join
            rc = v->s.add_miner(conn);
            if (rc == MH_OK) v->miners.insert(conn);
            break;
        case 1: {  // Request from a client
            const int64_t id = v->s.submit(conn, (const uint8_t*)m.data.data(), m.data.size(), m.lower, m.upper);
            if (id < 0)  // nothing will ever answer it: the transport closes the client (Disconnected)
                rc = mh::set_error(MH_EREJECTED, id == MH_ERANGE ? "Request refused: Lower > Upper"
                                                                 : "Request refused: Data too long");
            break;
        }
        case 2: {  // Result from a miner
            mh_completion c;
            const int r = v->s.result(conn, m.hash, m.nonce, now_ns, &c);
            if (r < 0) {
                rc = r;
            } else if (r == 1) {
                v->out.emplace_back(c.client, mh::encode(2, nullptr, 0, 0, 0, c.hash, c.nonce));
            }
            break;
        }
        default:
            rc = mh::set_error(MH_EINVAL, "unknown message type");
    }
    // a rejected Result requeued its chunk: hand the work out again either way
    const int d = v->dispatch(now_ns);
    return rc ? rc : d;
}

int mh_server_lost(mh_server* v, int64_t conn, uint64_t now_ns) {
    if (!v) return mh::set_error(MH_EINVAL, "NULL server");
    std::lock_guard<std::mutex> lk(v->mu);
    if (v->miners.erase(conn)) {
        const int rc = v->s.remove_miner(conn);
        if (rc) return rc;
    } else {
        v->s.drop_client(conn);
        // writes still queued for a lost client are dropped
        for (auto it = v->out.begin(); it != v->out.end();)
            it = (it->first == conn) ? v->out.erase(it) : it + 1;
    }
    return v->dispatch(now_ns);
}

int mh_server_pop_write(mh_server* v, int64_t* conn, char* out, size_t cap, size_t* len) {
    if (!v || !conn) return mh::set_error(MH_EINVAL, "bad arguments");
    std::lock_guard<std::mutex> lk(v->mu);
    if (v->out.empty()) return 0;
    const auto& w = v->out.front();
    if (len) *len = w.second.size();
    if (!out || cap < w.second.size()) return mh::set_error(MH_EINVAL, "output buffer too small");
    *conn = w.first;
    memcpy(out, w.second.data(), w.second.size());
    v->out.pop_front();
    return 1;
}

int mh_server_stats(mh_server* v, mh_sched_stats* out) {
    if (!v || !out) return mh::set_error(MH_EINVAL, "bad arguments");
    v->s.stats(out);
    return MH_OK;
}

}  // extern "C"
