// fuzz_host.cpp -- randomized host-side checks of libminehip's CPU code
// (planner, scheduler, server loop, Go-JSON codec) built with
// -fsanitize=address,undefined by tests/test_host_sanitize.py.  No GPU code is
// linked: mh_search / mh_search_multi (used by message.cpp's miner handler)
// are test doubles below that report MH_ENODEV, like the real ones on a host
// without a device.
//
//   fuzz_host <seed> <iterations>     exit 0 = every invariant held
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <random>
#include <string>
#include <vector>

#include "../../bitcoin-miner_amd/csrc/msgcodec.hpp"
#include "../../bitcoin-miner_amd/csrc/plan.hpp"
#include "../../bitcoin-miner_amd/csrc/sched.hpp"
#include "../../include/minehip.h"
#include "../../include/minehip_server.h"

namespace mh {
int set_error(int code, const char*) { return code; }
}  // namespace mh

extern "C" int mh_search(int, const uint8_t*, size_t, uint64_t, uint64_t, uint64_t*, uint64_t*) {
    return MH_ENODEV;
}
extern "C" int mh_search_multi(const int*, int, const uint8_t*, size_t, uint64_t, uint64_t, uint64_t, uint64_t*,
                               uint64_t*) {
    return MH_ENODEV;
}

static int g_fail = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                         \
            return;                                                           \
        }                                                                     \
    } while (0)

static std::mt19937_64 rng;
static uint64_t rnd(uint64_t n) { return n ? rng() % n : 0; }

static const uint64_t kP10[20] = {1ull, 10ull, 100ull, 1000ull, 10000ull, 100000ull, 1000000ull, 10000000ull,
                                  100000000ull, 1000000000ull, 10000000000ull, 100000000000ull,
                                  1000000000000ull, 10000000000000ull, 100000000000000ull,
                                  1000000000000000ull, 10000000000000000ull, 100000000000000000ull,
                                  1000000000000000000ull, 10000000000000000000ull};

static uint64_t interesting_u64() {
    switch (rnd(6)) {
        case 0: return rng();
        case 1: return ~0ull - rnd(100000);
        case 2: return rnd(2000000);
        default: {
            const uint64_t c = kP10[rnd(20)];
            const uint64_t off = rnd(50000);
            return rnd(2) ? (c > off ? c - off : 0) : (c + off < c ? ~0ull : c + off);
        }
    }
}

// The digits fast_search writes for lane u, group g and innermost digit i of a fast piece (its
// per-run formatting of U, the group digits and the per-nonce digit, restated from fast_search.hip
// on the host), read back as a decimal number, must be the nonce its candidate formula reports,
// inside the piece -- for the last-digit layouts and the Early ones (interleaved lanes included).
static uint64_t spread(uint64_t x, uint32_t k, uint32_t w) {  // fast_search.hip spread()
    if (k >= 20u) return x;
    uint64_t lo = 0, q = 1;
    for (uint32_t j = 0; j < k; ++j) {
        lo += (x % 10u) * q;
        q *= 10u;
        x /= 10u;
    }
    for (uint32_t j = 0; j < w; ++j) q *= 10u;
    return x * q + lo;
}
static uint64_t g_fast_checked = 0, g_early_checked = 0;
static bool lanes_format_their_nonces(const mh::Prefix& pre, const mh::Piece& p) {
    const mh::FastArgs& a = p.fa;
    const bool early = a.mode >= 3;
    ++g_fast_checked;
    g_early_checked += early ? 1u : 0u;
    const uint32_t base = (a.mode % 3 == mh::kModePre) ? 64u : 0u;
    const uint32_t d = (uint32_t)p.digits;
    for (int probe = 0; probe < 4; ++probe) {
        const uint64_t lane = probe == 0 ? 0 : probe == 1 ? a.n_runs - 1u : rnd(a.n_runs);
        const uint64_t U = a.u_start + lane;
        const uint32_t g = (uint32_t)rnd(a.n_groups), i = (uint32_t)rnd(10);
        uint8_t b[128];
        for (uint32_t x = 0; x < 128; ++x) b[x] = (uint8_t)(a.blk[x >> 2] >> (24u - 8u * (x & 3u)));
        uint64_t u = U;
        for (uint32_t k = 0; k < a.n_hi; ++k, u /= 10u)
            b[a.hi_end - 1u - k - ((early && k >= a.hole) ? a.hole_w : 0u)] += (uint8_t)(u % 10u);
        uint32_t gq = g;
        for (uint32_t j = 0; j + 1u < a.L; ++j, gq /= 10u) {
            const uint32_t pos = early ? a.g_last - j - (j >= a.g_hole ? 1u : 0u) : a.lo_pos + (a.L - 2u - j);
            b[base + pos] += (uint8_t)(gq % 10u);
        }
        b[base + (early ? a.inner : a.lo_pos + a.L - 1u)] += (uint8_t)i;
        uint64_t n = 0;
        for (uint32_t x = 0; x < d; ++x) {
            const uint8_t c = b[pre.t + x];
            if (c < '0' || c > '9' || (x == 0 && c == '0' && d > 1)) return false;
            n = n * 10u + (uint64_t)(c - '0');
        }
        const uint64_t want = early ? spread(U, a.hole, a.hole_w) * a.u_mul + spread(g, a.g_hole, 1) * a.g_mul + i * a.i_mul
                                    : U * a.pow10L + (uint64_t)g * 10u + i;
        if (n != want || n < p.first || n - p.first >= p.count) return false;
    }
    return true;
}

// planner: pieces tile [lo, hi] in order, in-bounds shapes
static void fuzz_plan() {
    std::string msg(rnd(700), 'a');
    for (auto& ch : msg) ch = (char)rnd(256);
    uint64_t lo = interesting_u64(), hi = interesting_u64();
    if (lo > hi) std::swap(lo, hi);
    if (rnd(3) == 0) hi = lo + rnd(3000000) < lo ? ~0ull : lo + rnd(3000000);
    mh::Prefix pre;
    mh::absorb_prefix((const uint8_t*)msg.data(), msg.size(), &pre);
    mh::PlanOpts o;
    o.lower_digits = 1 + (int)rnd(5);
    o.min_lanes = rnd(2) ? 1 : (1ull << rnd(20));
    o.max_nonces_per_launch = 1ull + rnd(1ull << 33);
    if (rnd(2)) o.max_blocks = 1u + (uint32_t)rnd(1u << 17);
    const uint64_t max_gen = (uint64_t)std::min(o.max_blocks, mh::kMaxBlocksPerLaunch) * mh::kBlockThreads;
    o.generic_below = rnd(2) ? 0 : rnd(1ull << 21);
    o.early = (int)rnd(2);
    o.fine_tail = rnd(2) ? 0 : rnd(1ull << 29);
    uint64_t cur = lo;
    bool done = false, bad = false;
    size_t n = 0;
    mh::plan_search(pre, lo, hi, o, [&](const mh::Piece& p) {
        if (done || p.first != cur || p.count == 0 || p.count - 1 > hi - p.first) {
            bad = true;
            return false;
        }
        if (p.kind == 0) {
            const uint64_t R = kP10[p.L];
            // the launch caps hold, rounded up to one lane at most (an Early block always fits them)
            if (p.L < 1 || p.L > 5 || p.first % R || p.count % R || p.fa.n_runs == 0 ||
                (uint64_t)p.fa.n_runs * R != p.count || p.fa.n_hi + p.fa.L > 20 ||
                p.count > std::max<uint64_t>(o.max_nonces_per_launch, R) || p.fa.n_runs > max_gen ||
                !lanes_format_their_nonces(pre, p)) {
                bad = true;
                return false;
            }
        } else if (p.ga.first != p.first || p.ga.count != p.count ||
                   p.count > (uint64_t)mh::kMaxBlocksPerLaunch * mh::kBlockThreads) {
            bad = true;
            return false;
        }
        const uint64_t last = p.first + (p.count - 1);
        if (last == hi) done = true; else cur = last + 1;
        return ++n < 100000;  // tiny launch sizes over wide ranges: stop early
    });
    CHECK(!bad);
    CHECK(done || n == 100000);
}

// codec: arbitrary bytes never crash; encode -> decode -> encode is a fixed point
static void fuzz_codec() {
    std::string junk(rnd(300), ' ');
    for (auto& ch : junk) ch = (char)(rnd(4) ? " {}\":,0123456789TypeDataLowerUpperHashNonce\\u"[rnd(44)] : rnd(256));
    mh_message m;
    uint8_t data[512];
    (void)mh_msg_decode(junk.data(), junk.size(), &m, data, sizeof data);

    std::string d(rnd(200), ' ');
    for (auto& ch : d) ch = (char)rnd(256);
    const int64_t type = (int64_t)rnd(3);
    const uint64_t a = interesting_u64(), b = interesting_u64(), h = rng(), nn = rng();
    const std::string e1 = mh::encode(type, (const uint8_t*)d.data(), d.size(), a, b, h, nn);
    mh::Msg x;
    CHECK(mh::decode(e1.data(), e1.size(), &x));
    CHECK(x.type == type && x.lower == a && x.upper == b && x.hash == h && x.nonce == nn);
    const std::string e2 = mh::encode(x.type, (const uint8_t*)x.data.data(), x.data.size(), x.lower, x.upper, x.hash,
                                      x.nonce);
    // Go writes an invalid byte as \ufffd but a valid U+FFFD raw, so the
    // fixed point is reached after one decode; for ASCII data at once
    bool ascii = true;
    for (unsigned char ch : d) ascii = ascii && ch < 0x80;
    CHECK(!ascii || e1 == e2);
    mh::Msg x2;
    CHECK(mh::decode(e2.data(), e2.size(), &x2) && x2.data == x.data);
    CHECK(mh::encode(x2.type, (const uint8_t*)x2.data.data(), x2.data.size(), x2.lower, x2.upper, x2.hash,
                     x2.nonce) == e2);
    // truncations of a valid payload are rejected, never read past the end
    const size_t cut = rnd(e1.size());
    std::vector<char> t(e1.begin(), e1.begin() + (ptrdiff_t)cut);
    mh::Msg y;
    CHECK(!mh::decode(t.data(), t.size(), &y));
}

// scheduler: random joins / losses / submits / drops / results; completed
// chunks of a finished job tile its range exactly once
static void fuzz_sched() {
    mh_sched_opts o;
    o.init_chunk = 1 + rnd(5000);
    o.min_chunk = 1 + rnd(300);
    o.max_chunk = o.min_chunk + rnd(10000);
    o.target_ns = 1 + rnd(100000);
    mh::Scheduler s(o);
    std::map<int64_t, std::pair<uint64_t, uint64_t>> range;       // job -> [lo, hi]
    std::map<int64_t, std::vector<std::pair<uint64_t, uint64_t>>> got;
    std::map<int64_t, bool> cancelled;
    std::map<int64_t, mh_assignment> out;  // miner -> outstanding chunk
    std::vector<int64_t> miners;
    int64_t next_miner = 0;
    uint64_t now = 0;
    for (int step = 0; step < 400; ++step) {
        now += 1 + rnd(1000);
        switch (rnd(8)) {
            case 0:
                if (s.add_miner(next_miner) == MH_OK) miners.push_back(next_miner);
                ++next_miner;
                break;
            case 1:
                if (!miners.empty()) {
                    const size_t i = rnd(miners.size());
                    CHECK(s.remove_miner(miners[i]) == MH_OK);
                    out.erase(miners[i]);
                    miners.erase(miners.begin() + (ptrdiff_t)i);
                }
                break;
            case 2: {
                uint64_t lo = interesting_u64(), hi;
                hi = lo + rnd(20000);
                if (hi < lo) hi = ~0ull;
                const int64_t j = s.submit((int64_t)rnd(5), (const uint8_t*)"m", 1, lo, hi);
                CHECK(j >= 0);
                range[j] = {lo, hi};
                break;
            }
            case 3: {
                const int64_t c = (int64_t)rnd(5);
                s.drop_client(c);
                break;
            }
            default: {
                mh_assignment a;
                const int r = s.next(-1, now, &a);
                CHECK(r == 0 || r == 1);
                if (r == 1) {
                    CHECK(out.find(a.miner) == out.end());
                    CHECK(range.count(a.job) && a.lower <= a.upper && a.lower >= range[a.job].first &&
                          a.upper <= range[a.job].second);
                    out[a.miner] = a;
                }
                if (!out.empty() && rnd(2)) {
                    auto it = out.begin();
                    std::advance(it, (long)rnd(out.size()));
                    const mh_assignment q = it->second;
                    out.erase(it);
                    const uint64_t nonce = q.lower + rnd(q.upper - q.lower + 1);
                    mh_completion c;
                    const int rr = s.result(q.miner, rng(), nonce, now, &c);
                    CHECK(rr == 0 || rr == 1);
                    got[q.job].push_back({q.lower, q.upper});
                    if (rr == 1) {
                        auto v = got[c.job];
                        std::sort(v.begin(), v.end());
                        uint64_t cur = range[c.job].first;
                        for (size_t k = 0; k < v.size(); ++k) {
                            CHECK(v[k].first == cur);
                            if (k + 1 < v.size()) cur = v[k].second + 1;
                        }
                        CHECK(!v.empty() && v.back().second == range[c.job].second);
                    }
                }
            }
        }
    }
    mh_sched_stats st;
    s.stats(&st);
    CHECK(st.miners == miners.size());
}

// server loop: arbitrary interleavings of payloads and losses never crash
static void fuzz_server() {
    mh_sched_opts o;
    mh_sched_default_opts(&o);
    o.init_chunk = o.min_chunk = 1 + rnd(1000);
    o.max_chunk = o.min_chunk + rnd(1000);
    mh_server* v = mh_server_create(&o);
    char buf[4096];
    for (int step = 0; step < 200; ++step) {
        const int64_t conn = (int64_t)rnd(8);
        std::string p;
        switch (rnd(5)) {
            case 0: p = mh::encode(0, nullptr, 0, 0, 0, 0, 0); break;
            case 1: p = mh::encode(1, (const uint8_t*)"cmu440", 6, interesting_u64(), interesting_u64(), 0, 0); break;
            case 2: p = mh::encode(2, nullptr, 0, 0, 0, rng(), interesting_u64()); break;
            case 3: mh_server_lost(v, conn, (uint64_t)step); continue;
            default: p = std::string(rnd(40), '{');
        }
        (void)mh_server_read(v, conn, p.data(), p.size(), (uint64_t)step);
        int64_t c;
        size_t n;
        while (mh_server_pop_write(v, &c, buf, sizeof buf, &n) == 1) {
            mh::Msg m;
            CHECK(mh::decode(buf, n, &m) && (m.type == 1 || m.type == 2));
        }
    }
    mh_server_destroy(v);
}

int main(int argc, char** argv) {
    const uint64_t seed = argc > 1 ? strtoull(argv[1], nullptr, 10) : 440;
    const int iters = argc > 2 ? atoi(argv[2]) : 200;
    rng.seed(seed);
    for (int i = 0; i < iters && !g_fail; ++i) {
        fuzz_plan();
        fuzz_codec();
        if (i % 4 == 0) fuzz_sched();
        if (i % 4 == 0) fuzz_server();
    }
    printf("fuzz_host seed=%llu iters=%d failures=%d fast_pieces=%llu early_pieces=%llu\n",
           (unsigned long long)seed, iters, g_fail, (unsigned long long)g_fast_checked,
           (unsigned long long)g_early_checked);
    return g_fail ? 1 : 0;
}
