// server_main.cpp -- minehip-server: the bitcoin server over LSP.
//
// Reference: bitcoin/server/server.go -- `server <port>` (:42-55), prints
// "Server listening on port <port>" (:58) and serves (:62, TODO in the
// reference).  The serving logic is libminehip's server
// loop (include/minehip_server.h: chunking by measured miner rate, lost-miner
// reassignment, lexicographic-min merge); this file only moves its messages
// over liblsp440 and reports lost connections to it (the N3 fix: the
// reference's lsp server never surfaces a lost client to Read).
#include <stdio.h>

#include <string>
#include <vector>

#include "../../../include/minehip.h"
#include "../../../include/minehip_server.h"
#include "common.hpp"

namespace {

// Upper bound of the LSP Data datagram that carries an n-byte payload: base64
// plus the JSON of lsp.Message with the largest ConnID / SeqNum / Size
// (lsp/message.go:17-24; {"Type":1,"ConnID":..,"SeqNum":..,"Size":..,"Payload":".."}).
size_t frame_bound(size_t n) { return 4 * ((n + 2) / 3) + 128; }

// A client Request is re-encoded for each miner chunk with other bounds (up to
// 20 digits each) and the server's own JSON escaping (Go's: <, >, & and control
// bytes as \u00XX, invalid UTF-8 as U+FFFD), so a Request that reached the
// server in one datagram need not fit in one as a miner Request.  Such a
// Request is refused up front: otherwise every chunk write would fail with
// LSP_ETOOBIG and the client would wait forever.
constexpr int64_t kRequest = 1;  // MsgType Request (message.go:9-13)

bool miner_request_fits(const uint8_t* payload, size_t n, std::vector<uint8_t>& scratch) {
    mh_message m;
    scratch.resize(3 * n + 16);  // an invalid UTF-8 byte decodes to U+FFFD, 3 bytes
    if (mh_msg_decode((const char*)payload, n, &m, scratch.data(), scratch.size()) != MH_OK || m.type != kRequest)
        return true;  // not a Request: the server loop decides what to do with it
    size_t need = 0;
    mh_msg_encode(kRequest, scratch.data(), m.data_len, UINT64_MAX, UINT64_MAX, 0, 0, nullptr, 0, &need);
    return frame_bound(need) <= LSP_MAX_DATAGRAM;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc != 2) {
        printf("Usage: ./%s <port>", argv[0]);  // server.go:42-45
        return 2;
    }
    uint64_t port = 0;
    if (!apps::parse_u64(argv[1], &port) || port > 65535) {
        printf("Port must be a number: %s\n", argv[1]);
        return 2;
    }
    const lsp_params p = apps::params_from_env();
    lsp_server* s = nullptr;
    const int rc = lsp_server_new((int)port, &p, &s);
    if (rc != LSP_OK) {
        printf("%s\n", apps::lsp_strerror(rc));
        return 1;
    }
    mh_sched_opts o;
    mh_sched_default_opts(&o);
    if (const char* e = getenv("MINEHIP_CHUNK")) {  // fixed chunk size (tests)
        o.init_chunk = o.min_chunk = o.max_chunk = strtoull(e, nullptr, 10);
    }
    mh_server* v = mh_server_create(&o);
    if (!v) {
        printf("bad MINEHIP_CHUNK\n");
        return 2;
    }
    printf("Server listening on port %d\n", lsp_server_port(s));
    fflush(stdout);

    std::vector<uint8_t> buf(1 << 16);
    std::vector<char> out(1 << 16);
    std::vector<uint8_t> scratch;
    for (;;) {
        int conn = 0;
        size_t n = 0;
        const int r = lsp_server_read(s, &conn, buf.data(), buf.size(), &n, -1);
        const uint64_t now = apps::now_ns();
        if (r == LSP_ESHORT) {
            buf.resize(n);
            continue;
        }
        if (r == LSP_OK) {
            // a refused Request gets no Result: close that client, which then prints
            // Disconnected; other bad payloads are ignored
            if (!miner_request_fits(buf.data(), n, scratch)) {
                fprintf(stderr, "minehip-server: conn %d: Request too large to forward to a miner in one "
                        "LSP datagram; refused\n", conn);
                lsp_server_close_conn(s, conn);
            } else if (mh_server_read(v, conn, (const char*)buf.data(), n, now) == MH_EREJECTED) {
                fprintf(stderr, "minehip-server: conn %d: %s\n", conn, mh_last_error());
                lsp_server_close_conn(s, conn);
            }
        } else if (conn != 0) {  // a client or miner lost / closed (server_api.go:7-17)
            mh_server_lost(v, conn, now);
            mh_sched_stats st;
            mh_server_stats(v, &st);
            fprintf(stderr, "minehip-server: conn %d %s; chunks requeued so far %llu\n", conn,
                    r == LSP_ELOST ? "lost" : "closed", (unsigned long long)st.chunks_requeued);
        } else {
            break;  // server closed
        }
        for (;;) {
            int64_t wc = 0;
            size_t wn = 0;
            const int k = mh_server_pop_write(v, &wc, out.data(), out.size(), &wn);
            if (k == MH_EINVAL) {
                out.resize(wn);
                continue;
            }
            if (k != 1) break;
            // a lost conn surfaces via Read; a frame too large for one datagram cannot happen for a
            // Request that passed miner_request_fits, but if it does, that miner can never get this
            // chunk: drop it as lost, so its chunk goes back to the job instead of hanging it
            if (lsp_server_write(s, (int)wc, (const uint8_t*)out.data(), wn) == LSP_ETOOBIG) {
                fprintf(stderr, "minehip-server: conn %d: write of %zu bytes exceeds one LSP datagram; "
                        "dropping the connection\n", (int)wc, wn);
                mh_server_lost(v, wc, now);
                lsp_server_close_conn(s, (int)wc);
            }
        }
    }
    mh_server_destroy(v);
    lsp_server_close(s);
    return 0;
}
