/*
 * minehip_server.h -- the caller side of the nonce search: the bitcoin
 * server's scheduler, exported by libminehip.so.
 *
 * Reference: bitcoin/server/server.go:12-20 (the server owns an lsp.Server)
 * and :62 ("TODO: implement this!") -- a stub.  Its job, per the CMU 15-440
 * P1 handout the stub belongs to:
 *   - miners connect and send Join (bitcoin/message.go:47-49);
 *   - a client sends Request{Data, Lower, Upper} (message.go:27-34);
 *   - the server splits [Lower, Upper] into chunks, hands each chunk to an
 *     idle miner as a Request, and merges the miners' Results
 *     (message.go:38-44) by the lexicographic min of (Hash, Nonce) -- the same
 *     associative merge as the miner's scan (miner.go:33 spec);
 *   - when every chunk is back it writes Result to the client;
 *   - a lost miner's chunk is handed to another miner, a lost client's job
 *     is dropped (lsp/server_api.go:7-17: Read returns the lost connID).
 *
 * Two layers, both transport-agnostic (no sockets: the LSP transport stays the
 * reference's, lsp/server_api.go):
 *   mh_sched_*   the scheduling state machine (jobs, chunks, miners);
 *   mh_server_*  the server's message loop on top of it: feed it every
 *                (connID, payload) that lsp.Server.Read returns, or the lost
 *                connID, and write out what mh_server_pop_write yields.
 * Every call is thread-safe (one internal mutex per object).  Times are
 * caller-supplied monotonic nanoseconds, so the schedule is deterministic
 * under test.  Return codes are those of minehip.h (mh_last_error explains).
 */
#ifndef MINEHIP_SERVER_H
#define MINEHIP_SERVER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Chunk sizing.  A miner's chunk is rate x target_ns, where rate is the
 * miner's measured nonces/ns (EWMA over its completed chunks; init_chunk
 * before the first one), capped at a fair share of the work left
 * (remaining / (2 x miners): guided self-scheduling, so the tail of a job is
 * spread over every miner) and clamped to [min_chunk, max_chunk]. */
typedef struct mh_sched_opts {
    uint64_t init_chunk; /* default 2^30: ~33 ms on one MI355X              */
    uint64_t min_chunk;  /* default 2^24                                     */
    uint64_t max_chunk;  /* default 2^38                                     */
    uint64_t target_ns;  /* default 250 ms per chunk                         */
} mh_sched_opts;

/* Defaults as documented above. */
void mh_sched_default_opts(mh_sched_opts *o);

typedef struct mh_sched mh_sched;

/* NULL opts = defaults.  Returns NULL on bad options (min > max, zero sizes). */
mh_sched *mh_sched_create(const mh_sched_opts *opts);
void mh_sched_destroy(mh_sched *s);

/* A miner joined (message.go:47 Join).  MH_EINVAL if the id is already known. */
int mh_sched_add_miner(mh_sched *s, int64_t miner);

/* A miner was lost: its outstanding chunk goes back to the front of its job.
 * MH_EINVAL if the id is unknown. */
int mh_sched_remove_miner(mh_sched *s, int64_t miner);

/* A client's Request: returns the new job id (>= 0) or MH_E*. */
int64_t mh_sched_submit(mh_sched *s, int64_t client, const uint8_t *msg, size_t len, uint64_t lower,
                        uint64_t upper);

/* A client was lost: its jobs are cancelled; chunks already out are ignored
 * when they come back.  Returns the number of jobs cancelled. */
int mh_sched_drop_client(mh_sched *s, int64_t client);

/* One chunk to send as a Request to a miner. */
typedef struct mh_assignment {
    int64_t miner, job;
    uint64_t lower, upper; /* inclusive */
    size_t msg_len;        /* the job's Data: mh_sched_job_msg */
} mh_assignment;

/* Hand one chunk to an idle miner: `miner` = a specific miner, or -1 for
 * any idle one (miners in join order; jobs served round-robin in submission
 * order).  Returns 1 and fills *out, or 0 when no idle miner / no pending
 * chunk. */
int mh_sched_next(mh_sched *s, int64_t miner, uint64_t now_ns, mh_assignment *out);

/* Copy job `job`'s Data into buf (cap bytes); *len receives its size. */
int mh_sched_job_msg(mh_sched *s, int64_t job, uint8_t *buf, size_t cap, size_t *len);

/* A job whose every chunk is back. */
typedef struct mh_completion {
    int64_t job, client;
    uint64_t hash, nonce;
} mh_completion;

/* A miner's Result for its outstanding chunk.  Returns 1 when that finished
 * its job (*out filled), 0 otherwise.  MH_EINVAL: the miner has no chunk out;
 * MH_ERANGE: nonce outside the chunk (the chunk is requeued, the miner idle). */
int mh_sched_result(mh_sched *s, int64_t miner, uint64_t hash, uint64_t nonce, uint64_t now_ns,
                    mh_completion *out);

typedef struct mh_sched_stats {
    uint64_t miners, idle_miners;
    uint64_t jobs;           /* live (incl. cancelled with chunks still out) */
    uint64_t chunks_assigned, chunks_done, chunks_requeued;
    uint64_t nonces_done;    /* nonces of completed chunks */
    uint64_t jobs_done, jobs_cancelled;
} mh_sched_stats;

int mh_sched_stats_read(mh_sched *s, mh_sched_stats *out);

/* ---- the server loop (server.go:62 TODO) ------------------------------ */

typedef struct mh_server mh_server;

mh_server *mh_server_create(const mh_sched_opts *opts);
void mh_server_destroy(mh_server *v);

/* lsp.Server.Read returned (conn, payload, nil).  Join registers a miner,
 * Request submits a job for the client `conn`, Result completes the miner's
 * chunk.  Queues the resulting writes.  MH_EINVAL for a payload that is not a
 * Message, or a Result from a connection with no chunk out.  MH_EREJECTED for
 * a client Request that can never be answered (Lower > Upper, Data longer
 * than MH_MAX_MSG_LEN): nothing is queued, and the caller should close that
 * connection (lsp.Server.CloseConn) so the client sees it end instead of
 * waiting forever for a Result. */
int mh_server_read(mh_server *v, int64_t conn, const char *payload, size_t len, uint64_t now_ns);

/* lsp.Server.Read returned (conn, nil, err): the connection is lost. */
int mh_server_lost(mh_server *v, int64_t conn, uint64_t now_ns);

/* Next queued lsp.Server.Write(conn, payload): returns 1 and fills it, 0 when
 * the queue is empty, MH_EINVAL when cap is short (*len = needed size; the
 * write stays queued). */
int mh_server_pop_write(mh_server *v, int64_t *conn, char *out, size_t cap, size_t *len);

int mh_server_stats(mh_server *v, mh_sched_stats *out);

#ifdef __cplusplus
}
#endif

#endif /* MINEHIP_SERVER_H */
