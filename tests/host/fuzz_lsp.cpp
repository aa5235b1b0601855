// fuzz_lsp.cpp -- liblsp440 (bitcoin-miner_amd/csrc/lsp/lsp.cpp) under
// sanitizers, built by tests/test_host_sanitize.py twice: with
// -fsanitize=address,undefined and with -fsanitize=thread (the Go reference's
// tests run under `go test -race`; this is the C++ counterpart).
//
//   fuzz_lsp <seed> <iterations>     exit 0 = every invariant held
//
// 1. codec: random and mutated datagrams into lsp_unmarshal (must not
//    crash), marshal -> unmarshal round trips of random messages;
// 2. endpoints: one server and several client threads echoing random
//    payloads over 127.0.0.1 with datagram loss and payload mangling, then
//    CloseConn / Close / lost-client reporting.
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lsp440.h"

static std::atomic<int> g_fail{0};
#define CHECK(c)                                                                  \
    do {                                                                          \
        if (!(c)) {                                                               \
            fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
            g_fail++;                                                             \
        }                                                                         \
    } while (0)

static void codec(std::mt19937_64& rng, int iters) {
    std::vector<uint8_t> pay(4096);
    char out[16384];
    for (int it = 0; it < iters * 20; ++it) {
        const size_t n = rng() % 600;
        std::string p;
        for (size_t i = 0; i < n; ++i) p.push_back((char)(rng() & 0xFF));
        const int type = (int)(rng() % 3);
        const int64_t conn = (int64_t)(rng() % 100000), seq = (int64_t)(rng() % 100000);
        const int has = (int)(rng() & 1) | (n > 0);
        size_t len = 0;
        CHECK(lsp_marshal(type, conn, seq, (int64_t)n, (const uint8_t*)p.data(), n, has, out, sizeof out, &len) ==
              LSP_OK);
        int t2 = -1, h2 = -1;
        int64_t c2 = -1, s2 = -1, z2 = -1;
        size_t pl = 0;
        CHECK(lsp_unmarshal(out, len, &t2, &c2, &s2, &z2, pay.data(), pay.size(), &pl, &h2) == LSP_OK);
        CHECK(t2 == type && c2 == conn && s2 == seq && z2 == (int64_t)n && h2 == has && pl == n);
        CHECK(pl == 0 || !memcmp(pay.data(), p.data(), n));
        // mutations: flip, cut, insert -> any result, no crash
        std::string m(out, len);
        for (int k = 0; k < 8; ++k) {
            std::string x = m;
            switch (rng() % 3) {
                case 0: if (!x.empty()) x[rng() % x.size()] = (char)(rng() & 0xFF); break;
                case 1: x.resize(rng() % (x.size() + 1)); break;
                default: x.insert(rng() % (x.size() + 1), 1, "{}[]\":,\\0aZ=-"[rng() % 14]); break;
            }
            (void)lsp_unmarshal(x.data(), x.size(), &t2, &c2, &s2, &z2, pay.data(), pay.size(), &pl, &h2);
        }
        std::string r;
        for (size_t i = 0; i < rng() % 64; ++i) r.push_back((char)(rng() & 0xFF));
        (void)lsp_unmarshal(r.data(), r.size(), &t2, &c2, &s2, &z2, pay.data(), pay.size(), &pl, &h2);
    }
}

static void endpoints(std::mt19937_64& rng, int round) {
    lsp_params p{20, 10, 1 + (int)(rng() % 5)};
    lsp_server* s = nullptr;
    CHECK(lsp_server_new(0, &p, &s) == LSP_OK);
    if (!s) return;
    const int port = lsp_server_port(s);
    std::atomic<bool> stop{false};
    std::thread echo([&] {
        std::vector<uint8_t> b(1 << 16);
        for (;;) {
            int c = 0;
            size_t n = 0;
            const int rc = lsp_server_read(s, &c, b.data(), b.size(), &n, 50);
            if (rc == LSP_ETIMEOUT) {
                if (stop) return;
                continue;
            }
            if (rc == LSP_OK) lsp_server_write(s, c, b.data(), n);
            else if (c == 0) return;
        }
    });
    const int nclients = 2 + round % 3;
    lsp_set_drop_percent(10, 10, 10, 10);
    lsp_set_msg_mangle_percent(10, 10);
    std::vector<std::thread> ts;
    const std::string hp = "127.0.0.1:" + std::to_string(port);
    for (int k = 0; k < nclients; ++k) {
        const uint64_t seed = rng();
        ts.emplace_back([&, k, seed] {
            std::mt19937_64 r(seed);
            lsp_client* c = nullptr;
            if (lsp_client_new(hp.c_str(), &p, &c) != LSP_OK) {
                CHECK(!"connect");
                return;
            }
            std::vector<std::string> msgs;
            for (int i = 0; i < 12; ++i) {
                std::string m = std::to_string(k) + ":" + std::to_string(i) + ":";
                for (size_t j = 0; j < r() % 200; ++j) m.push_back((char)(r() & 0xFF));
                msgs.push_back(m);
                CHECK(lsp_client_write(c, (const uint8_t*)m.data(), m.size()) == LSP_OK);
            }
            std::vector<uint8_t> b(1 << 16);
            for (auto& m : msgs) {
                size_t n = 0;
                const int rc = lsp_client_read(c, b.data(), b.size(), &n, 20000);
                CHECK(rc == LSP_OK && n == m.size() && !memcmp(b.data(), m.data(), n));
                if (rc != LSP_OK) break;
            }
            CHECK(lsp_client_conn_id(c) >= 1);
            CHECK(lsp_client_close(c) == LSP_OK);
        });
    }
    for (auto& t : ts) t.join();
    lsp_set_drop_percent(0, 0, 0, 0);
    lsp_set_msg_mangle_percent(0, 0);
    stop = true;
    echo.join();
    // clients that closed before their last acks got through are lost with
    // echoes unacked: Close reports that (server_api.go:31-37)
    const int crc = lsp_server_close(s);
    CHECK(crc == LSP_OK || crc == LSP_ELOST);
    // lost-client reporting: a client that closes is reported lost to Read
    CHECK(lsp_server_new(0, &p, &s) == LSP_OK);
    lsp_client* c = nullptr;
    const std::string hp2 = "127.0.0.1:" + std::to_string(lsp_server_port(s));
    CHECK(lsp_client_new(hp2.c_str(), &p, &c) == LSP_OK);
    const int id = lsp_client_conn_id(c);
    CHECK(lsp_client_write(c, (const uint8_t*)"x", 1) == LSP_OK);
    CHECK(lsp_client_close(c) == LSP_OK);
    int got = -1;
    uint8_t b[8];
    size_t n = 0;
    CHECK(lsp_server_read(s, &got, b, sizeof b, &n, 5000) == LSP_OK && got == id && n == 1);
    CHECK(lsp_server_read(s, &got, b, sizeof b, &n, 5000) == LSP_ELOST && got == id);
    CHECK(lsp_server_write(s, id, b, 1) == LSP_ELOST);
    CHECK(lsp_server_close(s) == LSP_OK);
}

int main(int argc, char** argv) {
    const uint64_t seed = argc > 1 ? strtoull(argv[1], nullptr, 10) : 440;
    const int iters = argc > 2 ? atoi(argv[2]) : 100;
    std::mt19937_64 rng(seed);
    codec(rng, iters);
    for (int r = 0; r < 3; ++r) endpoints(rng, r);
    printf("failures=%d\n", g_fail.load());
    return g_fail ? 1 : 0;
}
