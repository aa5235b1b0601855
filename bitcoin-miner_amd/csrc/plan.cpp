// plan.cpp -- see plan.hpp.
#include "plan.hpp"

#include <string.h>

#include <algorithm>
#include <cmath>

namespace mh {
namespace {

constexpr uint32_t kK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
constexpr uint32_t kIV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                             0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

inline uint32_t ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

constexpr uint64_t kPow10[20] = {1ull,
                                 10ull,
                                 100ull,
                                 1000ull,
                                 10000ull,
                                 100000ull,
                                 1000000ull,
                                 10000000ull,
                                 100000000ull,
                                 1000000000ull,
                                 10000000000ull,
                                 100000000000ull,
                                 1000000000000ull,
                                 10000000000000ull,
                                 100000000000000ull,
                                 1000000000000000ull,
                                 10000000000000000ull,
                                 100000000000000000ull,
                                 1000000000000000000ull,
                                 10000000000000000000ull};

// big-endian byte i of a 32-word tail image
inline void put_byte(uint32_t* w, uint32_t pos, uint32_t v) { w[pos >> 2] |= v << (24u - 8u * (pos & 3u)); }

void schedule(const uint32_t w16[16], uint32_t w[64]) {
    for (int i = 0; i < 16; ++i) w[i] = w16[i];
    for (int i = 16; i < 64; ++i) {
        const uint32_t s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3);
        const uint32_t s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
}

}  // namespace

int decimal_digits(uint64_t n) {
    int d = 1;
    while (d < 20 && n >= kPow10[d]) ++d;
    return d;
}

void host_compress(uint32_t st[8], const uint32_t w16[16]) {
    uint32_t w[64];
    schedule(w16, w);
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; ++i) {
        const uint32_t t1 = h + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + kK[i] + w[i];
        const uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1;
        d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

void absorb_prefix(const uint8_t* msg, size_t len, Prefix* out) {
    memcpy(out->mid, kIV, sizeof kIV);
    out->plen = (uint64_t)len + 1u;
    const uint64_t nfull = out->plen / 64u;
    uint32_t w[16];
    for (uint64_t blk = 0; blk < nfull; ++blk) {
        for (int i = 0; i < 16; ++i) {
            uint32_t v = 0;
            for (int k = 0; k < 4; ++k) {
                const uint64_t p = blk * 64u + (uint64_t)(4 * i + k);
                const uint32_t byte = (p < len) ? msg[p] : (uint32_t)' ';
                v = (v << 8) | byte;
            }
            w[i] = v;
        }
        host_compress(out->mid, w);
    }
    out->t = (uint32_t)(out->plen % 64u);
    memset(out->tail, 0, sizeof out->tail);
    for (uint32_t i = 0; i < out->t; ++i) {
        const uint64_t p = nfull * 64u + i;
        out->tail[i] = (p < len) ? msg[p] : (uint8_t)' ';
    }
}

void make_gen_args(const Prefix& pre, GenArgs* ga) {
    memset(ga, 0, sizeof *ga);
    memcpy(ga->mid, pre.mid, sizeof pre.mid);
    for (uint32_t i = 0; i < pre.t; ++i) put_byte(ga->tail, i, pre.tail[i]);
    ga->plen = pre.plen;
    ga->t = pre.t;
}

NonceCost nonce_cost(int J, int mode) {
    // Two counts of the same work:
    //   ops   VALU instructions with gfx950's 3-input ops (v_alignbit, v_bitop3, v_add3);
    //   slots issue slots of a SIMD-32 (2 cycles per wave64): full-rate ops
    //         (v_bitop3, 2-input adds, shifts) take 1, v_alignbit takes 2, and a
    //         sum costs one slot per addition (v_add3: 2 slots, 2 additions).
    // nonce-level words: those depending on word J (same rule as the kernel)
    uint64_t dep = 1ull << J;
    for (int t = 16; t < 64; ++t)
        if (((dep >> (t - 2)) | (dep >> (t - 7)) | (dep >> (t - 15)) | (dep >> (t - 16))) & 1ull) dep |= 1ull << t;
    auto is = [&](int t) { return (dep >> t) & 1ull; };
    uint32_t ops = 0, slots = 0;
    for (int t = 16; t < 64; ++t) {
        if (!is(t)) continue;
        // sigma: 2 alignbit + shift + xor3 (4 ops, 6 slots); a sum of n terms:
        // ceil((n-1)/2) add3 ops, n-1 slots
        const int s0 = (int)is(t - 15), s1 = (int)is(t - 2), a16 = (int)is(t - 16), a7 = (int)is(t - 7);
        const int hoisted = (s0 && s1 && a16 && a7) ? 0 : 1;  // group/run-level partial sum
        const int terms = s0 + s1 + a16 + a7 + hoisted;
        // sigma(W[J]) = sigma(wJ) ^ sigma(digit): one xor (the last digit never carries)
        const bool x0 = s0 && t - 15 == J, x1 = s1 && t - 2 == J;
        ops += (uint32_t)((s0 ? (x0 ? 1 : 4) : 0) + (s1 ? (x1 ? 1 : 4) : 0)) + (uint32_t)terms / 2u;
        slots += (uint32_t)((s0 ? (x0 ? 1 : 6) : 0) + (s1 ? (x1 ? 1 : 6) : 0)) + (uint32_t)(terms - 1);
    }
    // round J: T1 = hoisted + digit, e' and a' one add each
    ops += 3u;
    slots += 3u;
    // rounds J+1..63: 3+3 rotations, 2 xor3, Ch, Maj (16 slots) and the sums
    //   T1 = h + S1 + Ch + K + W (4 additions; 3 when K+W is hoisted, 2 when h+K+W is),
    //   e' = d + T1 (1), a' = T1 + S0 + Maj (2)
    for (int t = J + 1; t < 64; ++t) {
        const bool inv_w = !is(t), inv_h = inv_w && t <= J + 3;
        ops += inv_h ? 13u : 14u;
        slots += 16u + (inv_h ? 5u : inv_w ? 6u : 7u);
    }
    if (mode % 3 == kModeTwo) {
        ops += 8u;                   // feed-forward into block 1
        slots += 8u;
        ops += 64u * 14u - 1u;       // block 1: schedule host-known, no e' in its last round;
        slots += 64u * 22u - 1u;     // its last round also absorbs st0 (5 additions, 21 slots)
    } else {
        ops -= 1u;                   // last round: e' is dead, and K[63] + st0 rides in its sum
        slots -= 1u;
    }
    // H1 and the 64-bit compare run only on the rare new-best branch.
    ops += 2u;                       // last digit into W[J], compare H0
    slots += 2u;
    return NonceCost{ops, slots};
}

uint32_t nonce_ops(int J, int mode) { return nonce_cost(J, mode).ops; }

namespace {

// The instantiated fast kernels (layout.hpp MH_FAST_KERNELS, the launcher's list too).
bool kernel_exists(int J, int mode) { return fast_kernel_exists(J, mode); }

// Fast-kernel launch template for bucket d with L lower digits.  early: the digit ending the word
// before the last digit's is enumerated innermost (layout.hpp kMode*Early) -- false when the
// layout does not allow it.  *block_out: the nonces of one block of lanes, the unit a piece is cut
// in: 10^L, or for an Early layout 10^(p+L) (p: the innermost digit's decimal position).
bool make_fast_args(const Prefix& pre, int d, int L, bool early, int* J_out, int* mode_out, int* blocks_out,
                    uint64_t* block_out, FastArgs* fa) {
    const uint32_t t = pre.t;
    const uint32_t total = t + (uint32_t)d;
    const int nb = (total + 9u <= 64u) ? 1 : 2;
    const uint32_t pl = total - 1u;  // tail byte of the last digit
    int mode;
    uint32_t base;
    if (nb == 1) {
        mode = kModeOne;
        base = 0;
    } else if (pl >= 64u) {
        mode = kModePre;
        base = 64;
        // every enumerated digit must sit in block 1 (the Early layouts check theirs below)
        if (!early && pl - (uint32_t)L + 1u < 64u) return false;
    } else {
        mode = kModeTwo;
        base = 0;
    }
    const uint32_t lo = pl - (uint32_t)L + 1u - base;  // first lower digit, per-nonce-block relative
    int J = (int)((pl - base) >> 2);
    uint32_t p = 0, ib = 0;  // early: the innermost digit's decimal position and tail byte
    if (!early) {
        if ((int)(lo >> 2) < J - 1) return false;  // lower digits must span words J-1..J only
    } else {
        if (J < 1) return false;
        ib = base + 4u * (uint32_t)J - 1u;  // the byte ending word J - 1
        if (ib < t || ib < base) return false;  // no digit there, or not in the per-nonce block
        p = pl - ib;
        if (p < 1u || p >= (uint32_t)d) return false;
        // the group digits right before the innermost one, in its word (positions p+1 .. p+L-1):
        // the group then changes word J-1 only and no schedule word is group-level
        if (L > 4 || p + (uint32_t)L > (uint32_t)d || ib - (uint32_t)(L - 1) < t || ib - (uint32_t)(L - 1) < base)
            return false;
        J -= 1;
        mode += 3;
    }
    if (!kernel_exists(J, mode)) return false;

    memset(fa, 0, sizeof *fa);
    memcpy(fa->mid, pre.mid, sizeof pre.mid);
    for (uint32_t i = 0; i < t; ++i) put_byte(fa->blk, i, pre.tail[i]);
    for (uint32_t i = 0; i < (uint32_t)d; ++i) put_byte(fa->blk, t + i, 0x30u);  // '0' in every digit byte
    put_byte(fa->blk, total, 0x80u);
    const uint64_t bits = (pre.plen + (uint64_t)d) * 8u;
    const int lw = nb * 16 - 2;
    fa->blk[lw] = (uint32_t)(bits >> 32);
    fa->blk[lw + 1] = (uint32_t)bits;
    fa->pow10L = kPow10[L];
    fa->hi_end = total - (uint32_t)L;
    fa->n_hi = (uint32_t)(d - L);
    fa->lo_pos = lo;
    fa->L = (uint32_t)L;
    fa->n_groups = (uint32_t)kPow10[L - 1];
    fa->mode = (uint32_t)mode;
    fa->hole = kNoHole;
    fa->g_hole = kNoHole;
    fa->hole_w = 1;
    fa->g_mul = 1;
    uint64_t block = kPow10[L];
    if (early) {
        fa->inner = ib - base;
        fa->i_mul = kPow10[p];
        // positions p..p+L-1 enumerated (p: per nonce, p+1..: the group), U around them: its low
        // p digits, then its high digits from position p+L; a block of 10^(p+L) nonces is 10^p
        // interleaved lanes
        fa->g_last = ib - 1u - base;
        fa->hi_end = total;
        fa->hole = p;
        fa->hole_w = (uint32_t)L;
        fa->u_mul = 1;
        fa->g_mul = kPow10[p + 1u];
        block = kPow10[p + (uint32_t)L];
    }
    *block_out = block;
    if (mode % 3 == kModeTwo) {
        uint32_t w[64];
        schedule(fa->blk + 16, w);
        for (int i = 0; i < 64; ++i) fa->kw1[i] = kK[i] + w[i];
    }
    *J_out = J;
    *mode_out = mode;
    *blocks_out = nb;
    return true;
}

// The layout of bucket d's nonces [A, B] at L lower digits: the last digit innermost, or (opt.early)
// the digit ending the word before the last digit's, when that makes a nonce cheaper and the range
// still holds two blocks of its lanes.  False when no fast kernel takes the bucket at this L.
bool pick_layout(const Prefix& pre, int d, int L, uint64_t A, uint64_t B, const PlanOpts& opt, int* J, int* mode,
                 int* nb, uint64_t* block, FastArgs* fa) {
    if (!make_fast_args(pre, d, L, false, J, mode, nb, block, fa)) return false;
    if (opt.early) {
        int Je, me, nbe;
        uint64_t be;
        FastArgs fe;
        // a launch holds whole blocks (emit_runs), so an Early block must fit the launch caps: the
        // caps are then kept exactly, rounded up only to one 10^L-nonce lane
        const uint64_t max_gen = (uint64_t)std::min(opt.max_blocks, kMaxBlocksPerLaunch) * kBlockThreads;
        if (make_fast_args(pre, d, L, true, &Je, &me, &nbe, &be, &fe) &&
            nonce_cost(Je, me).slots < nonce_cost(*J, *mode).slots && B - A >= 2u * be &&
            be <= opt.max_nonces_per_launch && be / kPow10[L] <= max_gen) {
            *J = Je;
            *mode = me;
            *nb = nbe;
            *block = be;
            *fa = fe;
        }
    }
    return true;
}

// The fast layout of bucket d's nonces [A, B] (A <= B, all of [lower, upper] that lies in the
// bucket): L as the planner picks it and its layout (pick_layout), or false when the bucket goes
// to the generic kernel.
bool bucket_layout(const Prefix& pre, int d, uint64_t A, uint64_t B, const PlanOpts& opt, int* L_out, int* J,
                   int* mode, int* nb, uint64_t* block, FastArgs* fa) {
    int L = std::min(opt.lower_digits, d - 1);
    L = std::min(L, 5);
    // A lane runs 10^L nonces serially: a bucket with few runs would leave
    // most SIMDs idle and end in a long tail, so shorten the runs until
    // the bucket has min_lanes of them (2^19: ~8 workgroups per CU, one generation of the grid).
    while (L > 1 && (B - A) / kPow10[L] + 1u < opt.min_lanes) --L;
    while (L >= 1 && !pick_layout(pre, d, L, A, B, opt, J, mode, nb, block, fa)) --L;
    *L_out = L;
    return L >= 1 && B - A >= opt.generic_below;
}

inline uint64_t bucket_lo(int d) { return d == 1 ? 0u : kPow10[d - 1]; }
inline uint64_t bucket_hi(int d) { return d == 20 ? ~(uint64_t)0 : kPow10[d] - 1u; }

}  // namespace

void cost_segments(const Prefix& pre, uint64_t lower, uint64_t upper, const PlanOpts& opt,
                   std::vector<CostSeg>* out) {
    out->clear();
    const int d_lo = decimal_digits(lower), d_hi = decimal_digits(upper);
    for (int d = d_lo; d <= d_hi; ++d) {
        const uint64_t A = std::max(lower, bucket_lo(d)), B = std::min(upper, bucket_hi(d));
        int L = 0, J = 0, mode = 0, nb = 1;
        uint64_t blk = 1;
        FastArgs fa;
        double per;
        bool steady = false;
        if (bucket_layout(pre, d, A, B, opt, &L, &J, &mode, &nb, &blk, &fa)) {
            steady = L == opt.lower_digits && (B - A) / kPow10[L] + 1u >= (1u << 21);
            // the fast kernel's issue slots per nonce, plus the per-run / per-group work that shorter
            // lanes amortise over fewer nonces (L = 2: ~3%, L = 1: ~6% per nonce)
            per = (double)nonce_cost(J, mode).slots * (1.0 + 0.03 * (double)(3 - std::min(L, 3)));
            // a bucket of few generations of workgroups ends in a drain only partly back-filled:
            // the one-GPU model measured configs[3]'s d = 7..9 buckets in an 8-GPU shard ~15-20%
            // over the steady rate (profiles/r04o_inproc_model.json)
            if (!steady) per *= kUnsteadyFactor;
        } else {
            // generic kernel: every nonce formatted and hashed from the midstate
            const int blocks = (pre.t + (uint32_t)d + 9u <= 64u) ? 1 : 2;
            per = (double)kGenericSlotsPerBlock * blocks;
        }
        out->push_back(CostSeg{A, B, per, steady});
    }
}

double unsteady_share(const std::vector<CostSeg>& segs, uint64_t lo, uint64_t hi) {
    double all = 0.0, unsteady = 0.0;
    for (const CostSeg& s : segs) {
        const uint64_t a = std::max(s.a, lo), b = std::min(s.b, hi);
        if (a > b) continue;
        const double c = ((double)(b - a) + 1.0) * s.per;
        all += c;
        if (!s.steady) unsteady += c;
    }
    return all > 0.0 ? unsteady / all : 0.0;
}

double segments_cost(const std::vector<CostSeg>& segs, uint64_t lo, uint64_t hi) {
    double c = 0.0;
    for (const CostSeg& s : segs) {
        const uint64_t a = std::max(s.a, lo), b = std::min(s.b, hi);
        if (a <= b) c += ((double)(b - a) + 1.0) * s.per;
    }
    return c;
}

void split_by_cost(const std::vector<CostSeg>& segs, const std::vector<double>& w, std::vector<Span>* out) {
    out->assign(w.size(), Span{0, 0, true});
    if (segs.empty() || w.empty()) return;
    using u128 = unsigned __int128;
    double wsum = 0.0;
    for (double x : w) wsum += std::max(0.0, x);
    double total = 0.0;
    for (const CostSeg& s : segs) total += ((double)(s.b - s.a) + 1.0) * s.per;
    const uint64_t lower = segs.front().a;
    const u128 n_all = (u128)(segs.back().b - lower) + 1u;
    // Cut k (k = 1..n-1) after the nonce where the cost so far reaches total x (w_0 + .. + w_{k-1}) /
    // wsum; positions are nonce counts from lower (integers, monotone, the last one n_all), so the
    // spans tile [lower, upper] exactly whatever the rounding of the costs.
    u128 prev = 0;
    double acc_w = 0.0;
    for (size_t k = 0; k < w.size(); ++k) {
        acc_w += std::max(0.0, w[k]);
        u128 pos;
        if (k + 1 == w.size() || wsum <= 0.0) {
            pos = (k + 1 == w.size()) ? n_all : prev;
        } else {
            double target = total * (acc_w / wsum), cum = 0.0;
            pos = n_all;
            for (const CostSeg& s : segs) {
                const double len = (double)(s.b - s.a) + 1.0, c = len * s.per;
                if (cum + c >= target) {
                    double n = std::floor((target - cum) / s.per);
                    n = std::min(std::max(n, 0.0), len);
                    pos = (u128)(s.a - lower) + (u128)n;
                    break;
                }
                cum += c;
            }
            if (pos > n_all) pos = n_all;
        }
        if (pos < prev) pos = prev;
        if (pos > prev) (*out)[k] = Span{(uint64_t)(lower + (prev)), (uint64_t)(lower + (pos - 1u)), false};
        prev = pos;
    }
}

void plan_search(const Prefix& pre, uint64_t lower, uint64_t upper, const PlanOpts& opt,
                 const std::function<bool(const Piece&)>& cb) {
    GenArgs gbase;
    make_gen_args(pre, &gbase);
    const int d_lo = decimal_digits(lower), d_hi = decimal_digits(upper);
    const uint64_t max_gen = (uint64_t)std::min(opt.max_blocks, kMaxBlocksPerLaunch) * kBlockThreads;

    // Generic pieces are coalesced across buckets (the generic kernel formats
    // every nonce itself): small buckets and the ragged edges next to them go
    // out as one launch instead of one launch + merge each.
    bool have_gen = false;
    uint64_t gen_a = 0, gen_b = 0;  // pending generic range, inclusive
    auto flush_generic = [&]() -> bool {
        if (!have_gen) return true;
        have_gen = false;
        Piece p;
        memset(&p, 0, sizeof p);
        p.first = gen_a;
        p.count = gen_b - gen_a + 1u;
        p.kind = 1;
        p.digits = decimal_digits(gen_a);
        p.blocks = ((pre.t + (uint32_t)decimal_digits(gen_b) + 9u) <= 64u) ? 1 : 2;
        p.ga = gbase;
        p.ga.first = gen_a;
        p.ga.count = p.count;
        return cb(p);
    };
    auto emit_generic = [&](uint64_t a, uint64_t b, int) -> bool {  // [a, b] inclusive, a <= b
        for (;;) {
            if (have_gen && gen_b - gen_a < max_gen - 1u && gen_b + 1u == a) {
                const uint64_t room = max_gen - 1u - (gen_b - gen_a);  // nonces the pending piece can take
                if (b - a < room) {
                    gen_b = b;
                    return true;
                }
                gen_b = a + (room - 1u);
                a = gen_b + 1u;
            }
            if (!flush_generic()) return false;
            const uint64_t left = b - a;
            const uint64_t cnt = (left >= max_gen - 1u) ? max_gen : left + 1u;
            have_gen = true;
            gen_a = a;
            gen_b = a + (cnt - 1u);
            if (cnt - 1u == left) return true;
            a += cnt;
        }
    };

    // blocks [ua, ub) of Bx nonces of bucket d, each 10^Lx-nonce lanes [ua * lpb, ub * lpb)
    auto emit_runs = [&](int d, unsigned __int128 ua, unsigned __int128 ub, uint64_t Bx, int Lx, int Jx, int modex,
                         int nbx, const FastArgs& fax) -> bool {
        const unsigned __int128 Rx = kPow10[Lx];
        const uint64_t lpb = Bx / (uint64_t)Rx;  // lanes per block
        uint64_t max_runs = std::min<uint64_t>(max_gen, opt.max_nonces_per_launch / (uint64_t)Rx);
        // whole blocks per launch; pick_layout takes an Early layout (lpb > 1) only when one block
        // fits the caps, so this rounds up only a cap below one 10^L-nonce lane
        max_runs = std::max<uint64_t>(lpb, max_runs / lpb * lpb);
        ua *= lpb;
        ub *= lpb;
        for (unsigned __int128 u = ua; u < ub;) {
            const unsigned __int128 left = ub - u;
            const uint64_t runs = (left > max_runs) ? max_runs : (uint64_t)left;
            Piece p;
            memset(&p, 0, sizeof p);
            p.first = (uint64_t)(u * Rx);
            p.count = (uint64_t)((unsigned __int128)runs * Rx);
            p.kind = 0;
            p.digits = d;
            p.L = Lx;
            p.J = Jx;
            p.mode = modex;
            p.blocks = nbx;
            p.fa = fax;
            { const NonceCost nc = nonce_cost(Jx, modex); p.ops = nc.ops; p.slots = nc.slots; }
            p.fa.u_start = (uint64_t)u;
            p.fa.n_runs = (uint32_t)runs;
            p.ga = gbase;
            if (!flush_generic() || !cb(p)) return false;
            u += runs;
        }
        return true;
    };
    // [a, b] (a <= b) of bucket d outside the whole blocks of an Early layout (< 10^(p+L) nonces
    // at each end): 10-nonce runs of the last-digit layout -- short workgroups, on the low-
    // priority stream, so that an edge never ends a search with a few 1,000-nonce lanes -- and
    // the ragged rest on the generic kernel
    auto emit_edge = [&](int d, uint64_t a, uint64_t b) -> bool {
        FastArgs fs;
        int Js = 0, ms = 0, nbs = 1;
        uint64_t bs = 1;
        const int L = 1;
        if (!make_fast_args(pre, d, L, false, &Js, &ms, &nbs, &bs, &fs)) return emit_generic(a, b, d);
        const unsigned __int128 R = bs;
        const unsigned __int128 u0 = ((unsigned __int128)a + R - 1u) / R, u1 = ((unsigned __int128)b + 1u) / R;
        if (u0 >= u1) return emit_generic(a, b, d);
        if (a < (uint64_t)(u0 * R) && !emit_generic(a, (uint64_t)(u0 * R) - 1u, d)) return false;
        if (!emit_runs(d, u0, u1, bs, L, Js, ms, nbs, fs)) return false;
        return u1 * R > (unsigned __int128)b || emit_generic((uint64_t)(u1 * R), b, d);
    };

    for (int d = d_lo; d <= d_hi; ++d) {
        const uint64_t A = std::max(lower, bucket_lo(d)), B = std::min(upper, bucket_hi(d));
        FastArgs fa;
        int L = 0, J = 0, mode = 0, nb = 1;
        uint64_t blk = 1;
        if (!bucket_layout(pre, d, A, B, opt, &L, &J, &mode, &nb, &blk, &fa)) {
            if (!emit_generic(A, B, d)) return;
            continue;
        }
        // whole blocks of lanes: a block is one run of 10^L nonces, or (an Early layout) the
        // 10^(p+L) nonces its 10^p lanes interleave; an Early layout's ragged ends go to the
        // last-digit layout's runs first (emit_edge)
        const bool early = mode >= 3;
        const unsigned __int128 R = blk;
        const unsigned __int128 U0 = ((unsigned __int128)A + R - 1u) / R;
        const unsigned __int128 U1p = ((unsigned __int128)B + 1u) / R;  // one past the last full block
        if (U0 >= U1p) {
            if (!(early ? emit_edge(d, A, B) : emit_generic(A, B, d))) return;
            continue;
        }
        const uint64_t fast_first = (uint64_t)(U0 * R);
        const unsigned __int128 fast_end = U1p * R;  // exclusive, may be 2^64
        if (A < fast_first && !(early ? emit_edge(d, A, fast_first - 1u) : emit_generic(A, fast_first - 1u, d)))
            return;
        // Tail split (opt.fine_tail): the last runs of a full-L bucket at L - 1, so that their
        // short workgroups can back-fill the drain of the coarse launches (streams = 2).
        unsigned __int128 U_split = U1p;  // coarse blocks [U0, U_split), then the tail at L - 1
        int Lf = 0, Jf = 0, modef = 0, nbf = 1;
        uint64_t blkf = 1;
        FastArgs faf;
        if (opt.fine_tail && L == opt.lower_digits && L >= 2) {
            const unsigned __int128 tail_blocks = opt.fine_tail / (uint64_t)R;
            if (tail_blocks >= 1 && (U1p - U0) > 4 * tail_blocks &&
                pick_layout(pre, d, L - 1, A, B, opt, &Jf, &modef, &nbf, &blkf, &faf) && R % blkf == 0u) {
                U_split = U1p - tail_blocks;
                Lf = L - 1;
            }
        }
        if (!emit_runs(d, U0, U_split, blk, L, J, mode, nb, fa)) return;
        if (U_split < U1p && !emit_runs(d, U_split * (R / blkf), U1p * (R / blkf), blkf, Lf, Jf, modef, nbf, faf))
            return;
        if (fast_end <= (unsigned __int128)B &&
            !(early ? emit_edge(d, (uint64_t)fast_end, B) : emit_generic((uint64_t)fast_end, B, d)))
            return;
    }
    flush_generic();
}

}  // namespace mh
