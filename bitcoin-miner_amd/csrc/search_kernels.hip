// search_kernels.hip -- gfx950 kernels of libminehip.
//
// Hot path replaced: the miner's scan over bitcoin.Hash (reference
// bitcoin/hash.go:13-17, scan spec SURVEY.md §8(a) A2 / stub
// bitcoin/miner/miner.go:33).  Design: DESIGN.md §3.
//
//   fast_search<J, MODE>  one lane = one run of 10^L consecutive nonces that
//                         share their d-L higher digits; the L lower digits
//                         are enumerated in wave-uniform loops (digit
//                         arithmetic is SALU); only message word J (the last
//                         digit's word) changes per nonce, so the compiler
//                         hoists rounds 0..J-1 and every schedule term that
//                         does not depend on W[J] out of the per-nonce loop.
//   generic_scan          one lane = one nonce, any layout (range edges,
//                         buckets too small for runs).
//   hash_batch            out[i] = Hash(msg, nonces[i]) (GPU bitcoin.Hash).
//   merge_partials        folds per-workgroup (hash, nonce) candidates into
//                         the search's running minimum (one 1024-thread
//                         workgroup).
//
// Every candidate comparison is the lexicographic (hash, nonce) order, which
// equals the reference loop's strict-< first minimum.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <map>
#include <mutex>
#include <string>

#include "layout.hpp"
#include "sha256_gfx950.hpp"

// minimum waves per SIMD the fast kernel is compiled for (register budget)
#ifndef MH_MIN_WAVES
#define MH_MIN_WAVES 1
#endif

namespace mh {
namespace dev {

__device__ __forceinline__ bool lex_less(uint64_t ha, uint64_t na, uint64_t hb, uint64_t nb) {
    return ha < hb || (ha == hb && na < nb);
}

// One exchange step of the wave reduction: the partner's (hash, nonce),
// fetched dword by dword by a DPP move (CTRL < 0x200: CTRL is the dpp_ctrl)
// or by a ds_swizzle (CTRL >= 0x200: the swizzle offset is CTRL - 0x200).
template <int CTRL>
__device__ __forceinline__ uint32_t xlane(uint32_t v) {
    if constexpr (CTRL < 0x200)
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
    else
        return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, CTRL - 0x200);
}

template <int CTRL>
__device__ __forceinline__ void wave_step(uint64_t& h, uint64_t& n) {
    const uint64_t oh = ((uint64_t)xlane<CTRL>((uint32_t)(h >> 32)) << 32) | xlane<CTRL>((uint32_t)h);
    const uint64_t on = ((uint64_t)xlane<CTRL>((uint32_t)(n >> 32)) << 32) | xlane<CTRL>((uint32_t)n);
    if (lex_less(oh, on, h, n)) {
        h = oh;
        n = on;
    }
}

// Workgroup lexicographic min; the result is valid in thread 0.
// Wave level: DPP quad_perm [1,0,3,2] and [2,3,0,1], row_half_mirror,
// row_mirror (each step joins two groups whose lanes already agree, so after
// it every lane of the doubled group holds its min), then ds_swizzle xor 16
// (bit mode, within 32 lanes), then lane 0 takes lane 32's value.  Then LDS
// across the workgroup's waves.
template <int NT = kBlockThreads>
__device__ __forceinline__ void block_min(uint64_t& h, uint64_t& n) {
    wave_step<0xB1>(h, n);              // quad_perm [1,0,3,2]: lane ^ 1
    wave_step<0x4E>(h, n);              // quad_perm [2,3,0,1]: lane ^ 2
    wave_step<0x141>(h, n);             // row_half_mirror: quads of 8 lanes
    wave_step<0x140>(h, n);             // row_mirror: halves of 16-lane rows
    wave_step<0x200 + 0x401F>(h, n);    // ds_swizzle and 0x1F, xor 0x10: rows 0<->1, 2<->3
    {
        const uint64_t oh = ((uint64_t)__builtin_amdgcn_readlane((int)(h >> 32), 32) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)h, 32);
        const uint64_t on = ((uint64_t)__builtin_amdgcn_readlane((int)(n >> 32), 32) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)n, 32);
        if (lex_less(oh, on, h, n)) {
            h = oh;
            n = on;
        }
    }
    __shared__ uint64_t sh[NT / 64], sn[NT / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0) {
        sh[wv] = h;
        sn[wv] = n;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 1; i < NT / 64; ++i)
            if (lex_less(sh[i], sn[i], h, n)) {
                h = sh[i];
                n = sn[i];
            }
    }
}

// w[wi] += v for a word index that is not a compile-time constant, without
// dynamic register indexing (which would go to scratch).
template <int NW>
__device__ __forceinline__ void add_word(uint32_t (&w)[NW], uint32_t wi, uint32_t v) {
#pragma unroll
    for (int x = 0; x < NW; ++x) w[x] += (wi == (uint32_t)x) ? v : 0u;
}

// Rounds of a block whose message schedule is fully known on the host:
// kw[i] = K[i] + W[i].  Returns only H0/H1 (feed-forward of words 0, 1).
__device__ __forceinline__ void sha256_block_kw_h01(const uint32_t st[8], const uint32_t* kw, uint32_t& h0,
                                                    uint32_t& h1) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        const uint32_t t1 = h + bsig1(e) + ch(e, f, g) + kw[i];
        const uint32_t t2 = bsig0(a) + maj(a, b, c);
        h = g; g = f; f = e; e = d + t1;
        d = c; c = b; b = a; a = t1 + t2;
    }
    h0 = st[0] + a;
    h1 = st[1] + b;
}

// Generic Hash(msg, n): formats n in registers and hashes the 1 or 2 tail
// blocks from the host midstate.  Handles any digit count per lane.
__device__ __forceinline__ void hash_generic(const GenArgs& a, uint64_t n, uint32_t& h0, uint32_t& h1) {
    constexpr uint64_t P10[20] = {1ull, 10ull, 100ull, 1000ull, 10000ull, 100000ull, 1000000ull, 10000000ull,
                                  100000000ull, 1000000000ull, 10000000000ull, 100000000000ull,
                                  1000000000000ull, 10000000000000ull, 100000000000000ull,
                                  1000000000000000ull, 10000000000000000ull, 100000000000000000ull,
                                  1000000000000000000ull, 10000000000000000000ull};
    uint32_t nd = 1;  // Go %d: no leading zeros, "0" for 0
#pragma unroll
    for (int k = 1; k < 20; ++k) nd += (n >= P10[k]) ? 1u : 0u;
    uint32_t w[32];
#pragma unroll
    for (int x = 0; x < 16; ++x) w[x] = a.tail[x];
#pragma unroll
    for (int x = 16; x < 32; ++x) w[x] = 0u;
    uint64_t u = n;
#pragma unroll
    for (int k = 0; k < 20; ++k) {
        if ((uint32_t)k < nd) {
            const uint64_t q = u / 10u;
            const uint32_t dg = (uint32_t)(u - q * 10u);
            u = q;
            const uint32_t pos = a.t + nd - 1u - (uint32_t)k;
            add_word(w, pos >> 2, (0x30u + dg) << (24u - 8u * (pos & 3u)));
        }
    }
    const uint32_t end = a.t + nd;  // tail length; the 0x80 byte goes here
    add_word(w, end >> 2, 0x80u << (24u - 8u * (end & 3u)));
    const uint64_t bits = (a.plen + nd) * 8u;
    const bool two = end + 9u > 64u;
    const uint32_t bhi = (uint32_t)(bits >> 32), blo = (uint32_t)bits;
    w[14] = two ? w[14] : bhi;
    w[15] = two ? w[15] : blo;
    w[30] = two ? bhi : 0u;
    w[31] = two ? blo : 0u;
    uint32_t st[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) st[i] = a.mid[i];
    if (!two) {
        sha256_block_h01(st, w, h0, h1);
    } else {
        sha256_block(st, w);
        sha256_block_h01(st, w + 16, h0, h1);
    }
}

}  // namespace dev

// ---------------------------------------------------------------------------
// fast_search<J, MODE>
// ---------------------------------------------------------------------------
// Inside a lane only message word J (the last digit's word) changes from one
// nonce to the next, and word J-1 changes once per group of 10 nonces.  Every
// schedule word W[t] therefore lives at one of three levels, fixed at compile
// time by J:
//   nonce  depends on W[J]                    -> computed per nonce
//   group  depends on W[J-1] but not on W[J]  -> once per 10 nonces
//   run    neither                            -> once per lane (10^L nonces)
// and each per-nonce / per-group word is split into its cheaper-level partial
// sum plus the terms of its own level.  Words after J hold only padding and
// length, so they come from the kernel arguments (SGPRs), never VGPRs.
// The hoisting is explicit: left to LICM it does not happen, because SROA
// turns the message array into a loop-carried vector.
struct Dep {
    static constexpr uint64_t from(int j) {  // words whose value depends on word j
        if (j < 0) return 0;
        uint64_t m = 1ull << j;
        for (int t = 16; t < 64; ++t)
            if (((m >> (t - 2)) | (m >> (t - 7)) | (m >> (t - 15)) | (m >> (t - 16))) & 1ull) m |= 1ull << t;
        return m;
    }
};

// sigma0/sigma1 of the last digit's contribution inc = i << 8k (i = 0..9,
// k = byte slot).  The last digit's byte of word J is '0' before the digit
// is added and 0x30 + i never carries, so W[J] = wJ ^ inc and, sigma being
// GF(2)-linear, sigma(W[J]) = sigma(wJ) ^ sigma(inc): one VALU xor per nonce
// with a scalar (SMEM) operand instead of four VALU ops.
struct IncSigma {
    uint32_t s0[4][10], s1[4][10];
};
constexpr uint32_t crotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
constexpr IncSigma make_inc_sigma() {
    IncSigma t{};
    for (int k = 0; k < 4; ++k)
        for (uint32_t i = 0; i < 10; ++i) {
            const uint32_t x = i << (8 * k);
            t.s0[k][i] = crotr(x, 7) ^ crotr(x, 18) ^ (x >> 3);
            t.s1[k][i] = crotr(x, 17) ^ crotr(x, 19) ^ (x >> 10);
        }
    return t;
}
static __constant__ IncSigma kIncSigma = make_inc_sigma();  // static: one copy per translation unit

namespace dev {
// Last round of a compression when only H0 = st0 + a64 is needed:
// kw_st0 = K[63] + W[63] + st0.  Seven terms, three add3.
__device__ __forceinline__ uint32_t last_round_h0(uint32_t a, uint32_t b, uint32_t c, uint32_t e, uint32_t f,
                                                  uint32_t g, uint32_t h, uint32_t kw_st0) {
    return ((h + kw_st0) + bsig1(e) + ch(e, f, g)) + (bsig0(a) + maj(a, b, c));
}

// Block whose schedule is host-known (kw[i] = K[i] + W[i]): H0 and a63.
__device__ __forceinline__ void sha256_block_kw_last(const uint32_t st[8], const uint32_t* kw, uint32_t& h0,
                                                     uint32_t& a63);

// One round; kw = K[t] + W[t].  (h + kw) first, so it folds into a single
// hoisted value whenever both are invariant.
__device__ __forceinline__ void round_kw(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t& e,
                                         uint32_t& f, uint32_t& g, uint32_t& h, uint32_t kw) {
    const uint32_t t1 = (h + kw) + bsig1(e) + ch(e, f, g);
    const uint32_t t2 = bsig0(a) + maj(a, b, c);
    h = g; g = f; f = e; e = d + t1;
    d = c; c = b; b = a; a = t1 + t2;
}

__device__ __forceinline__ void sha256_block_kw_last(const uint32_t st[8], const uint32_t* kw, uint32_t& h0,
                                                     uint32_t& a63) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int i = 0; i < 63; ++i) round_kw(a, b, c, d, e, f, g, h, kw[i]);
    a63 = a;
    h0 = last_round_h0(a, b, c, e, f, g, h, kw[63] + st[0]);
}
}  // namespace dev

template <int J, int MODE>
__global__ __launch_bounds__(kBlockThreads, MH_MIN_WAVES) void fast_search(const FastArgs a,
                                                                           Partial* __restrict__ partials) {
    using namespace dev;
    constexpr uint32_t K[64] = MH_K256;
    constexpr uint64_t NM = Dep::from(J);               // nonce-level words
    constexpr uint64_t GM = Dep::from(J - 1) & ~NM;     // group-level words
    constexpr int BASE = (MODE == kModePre) ? 16 : 0;   // per-nonce block inside the tail
#define MH_N(t) ((NM >> (t)) & 1ull)
#define MH_G(t) ((GM >> (t)) & 1ull)
#define MH_R(t) (!MH_N(t) && !MH_G(t))
    const uint32_t gid = blockIdx.x * kBlockThreads + threadIdx.x;
    const uint64_t U = a.u_start + gid;

    // ---- per run --------------------------------------------------------
    // Tail words: host template + the d-L digits of U, right-aligned so U's
    // last digit sits at tail byte hi_end-1.  Only words before the lower
    // digits can receive them (words < BASE + J).
    constexpr int NW = BASE + J + 1;
    uint32_t w[NW];
#pragma unroll
    for (int x = 0; x < NW; ++x) w[x] = a.blk[x];
    {
        uint64_t u = U;
#pragma unroll
        for (int k = 0; k < 20; ++k) {
            if ((uint32_t)k < a.n_hi) {
                const uint64_t q = u / 10u;
                const uint32_t dg = (uint32_t)(u - q * 10u);
                u = q;
                const uint32_t pos = a.hi_end - 1u - (uint32_t)k;
                add_word(w, pos >> 2, dg << (24u - 8u * (pos & 3u)));
            }
        }
    }
    // words of the per-nonce block: per-lane up to J, uniform (SGPR) after J
    uint32_t W[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) W[t] = (t <= J) ? w[BASE + t] : a.blk[BASE + t];

    uint32_t st[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) st[i] = a.mid[i];
    if constexpr (MODE == kModePre) {
        uint32_t b0[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) b0[t] = w[t];
        sha256_block(st, b0);  // tail block 0 holds no lower digit: once per run
    }
    // rounds 0..J-2 read only run-level words
    uint32_t ra = st[0], rb = st[1], rc = st[2], rd = st[3], re = st[4], rf = st[5], rg = st[6], rh = st[7];
#pragma unroll
    for (int t = 0; t + 1 < J; ++t) round_kw(ra, rb, rc, rd, re, rf, rg, rh, K[t] + W[t]);

    // run-level schedule words, and the run-level part of the others
    uint32_t wr[64], pr[64];
#pragma unroll
    for (int t = 0; t < 16; ++t) wr[t] = W[t];
#pragma unroll
    for (int t = 16; t < 64; ++t) {
        uint32_t v = 0u;
        if (MH_R(t - 16)) v += wr[t - 16];
        if (MH_R(t - 7)) v += wr[t - 7];
        if (MH_R(t - 15)) v += ssig0(wr[t - 15]);
        if (MH_R(t - 2)) v += ssig1(wr[t - 2]);
        if (MH_R(t)) wr[t] = v; else pr[t] = v;
    }
    // K[t] + W[t] of the run-level words the per-nonce rounds read, made
    // opaque so the register allocator keeps the sums instead of redoing the
    // add on every nonce (it did, for t = 16..18, once the lane's best moved
    // to SGPRs and freed VGPRs).
    uint32_t kwr[64];
#pragma unroll
    for (int t = 16; t < 64; ++t)
        if (MH_R(t) && t > J) {
            kwr[t] = K[t] + wr[t];
            asm volatile("" : "+v"(kwr[t]));
        }

    const uint32_t lastpos = a.lo_pos + a.L - 1u;  // byte of the last digit, in word J
    const uint32_t sh_last = 24u - 8u * (lastpos & 3u);
    // The best (H0, H1, nonce) of the whole wave so far, wave-uniform (SGPRs).
    // A lane is a candidate when its H0 <= the wave's best H0: the compare is
    // already a lane mask, and the scan over its set bits is scalar work.
    // Per wave, the candidate branch is taken ~ln(steps) times per run; per
    // lane it was taken whenever any of 64 lanes improved its own minimum,
    // ~64 + 64 ln(steps / 64) times, i.e. on ~93% of the steps of a 100-nonce
    // run.  Invalid lanes (gid >= n_runs) never become candidates.
    const uint64_t valid_mask = __builtin_amdgcn_ballot_w64(gid < a.n_runs);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t wave_u0 = a.u_start + (uint64_t)blockIdx.x * kBlockThreads + wave * 64u;
    uint32_t wbh0 = 0xFFFFFFFFu, wbh1 = 0xFFFFFFFFu;
    uint64_t wbn = ~0ull;

    for (uint32_t g = 0; g < a.n_groups; ++g) {
        // ---- per group of 10 nonces --------------------------------------
#if defined(MH_SYNC) && MH_SYNC == 10
        __builtin_amdgcn_s_barrier();
#endif
        // digits 0..L-2 of q = 10*g + i: wave-uniform, so this is SALU work
        uint32_t cj = 0u, cjm = 0u, gq = g;
        for (uint32_t k = a.L - 1u; k-- > 0u;) {
            const uint32_t q = gq / 10u;
            const uint32_t dg = gq - q * 10u;
            gq = q;
            const uint32_t p = a.lo_pos + k;
            const uint32_t v = dg << (24u - 8u * (p & 3u));
            if ((p >> 2) == (uint32_t)J)
                cj += v;
            else
                cjm += v;
        }
        const uint32_t wJ = W[J] + cj;  // word J with this group's digits, last digit '0'
        const uint32_t s0wJ = ssig0(wJ), s1wJ = ssig1(wJ);
        uint32_t wg[64], pg[64];
        if constexpr (J > 0) wg[J - 1] = W[J - 1] + cjm;
#pragma unroll
        for (int t = 16; t < 64; ++t) {
            if (MH_R(t)) continue;
            uint32_t v = pr[t];
            if (MH_G(t - 16)) v += wg[t - 16];
            if (MH_G(t - 7)) v += wg[t - 7];
            if (MH_G(t - 15)) v += ssig0(wg[t - 15]);
            if (MH_G(t - 2)) v += ssig1(wg[t - 2]);
            if (MH_G(t)) wg[t] = v; else pg[t] = v;
        }
        // round J-1 reads the group-level word J-1
        uint32_t ga = ra, gb = rb, gc = rc, gd = rd, ge = re, gf = rf, gG = rg, gh = rh;
        if constexpr (J > 0) round_kw(ga, gb, gc, gd, ge, gf, gG, gh, K[J - 1] + wg[J - 1]);
        // round J: every input but W[J]'s last digit is known here
        const uint32_t t1J = (gh + (K[J] + wJ)) + bsig1(ge) + ch(ge, gf, gG);
        const uint32_t t2J = bsig0(ga) + maj(ga, gb, gc);

        for (uint32_t i = 0; i < 10u; ++i) {
            // ---- per nonce ------------------------------------------------
#if defined(MH_SYNC) && MH_SYNC == 1
            __builtin_amdgcn_s_barrier();
#endif
            const uint32_t inc = i << sh_last;  // SALU
            const uint32_t s0inc = kIncSigma.s0[sh_last >> 3][i], s1inc = kIncSigma.s1[sh_last >> 3][i];
            uint32_t x[64];
            x[J] = wJ + inc;
            // schedule word t, computed right before the round that reads it rather
            // than all words first: the same instructions, but the AMDGPU scheduler
            // then emits an order that issues 1.8% faster on configs[1] and 1.5% on
            // the Pre-mode layouts (profiles/r01zz13_cur_vs_ildef.jsonl)
            auto sched = [&](int t) {
                if (t < 16 || !MH_N(t)) return;
                uint32_t v = pg[t];
                if (MH_N(t - 16)) v += x[t - 16];
                if (MH_N(t - 7)) v += x[t - 7];
                if (MH_N(t - 15)) v += (t - 15 == J) ? (s0wJ ^ s0inc) : ssig0(x[t - 15]);
                if (MH_N(t - 2)) v += (t - 2 == J) ? (s1wJ ^ s1inc) : ssig1(x[t - 2]);
                x[t] = v;
            };
            const uint32_t t1 = t1J + inc;
            uint32_t A = t1 + t2J, B = ga, C = gb, D = gc, E = gd + t1, F = ge, G = gf, H = gG;
            uint32_t h0, a63;
            if constexpr (MODE != kModeTwo) {
#pragma unroll
                for (int t = J + 1; t < 63; ++t) {
                    sched(t);
                    round_kw(A, B, C, D, E, F, G, H,
                             (t >= 16 && MH_R(t)) ? kwr[t] : K[t] + (MH_N(t) ? x[t] : (MH_G(t) ? wg[t] : wr[t])));
                }
                sched(63);
                a63 = A;
                h0 = last_round_h0(A, B, C, E, F, G, H,
                                   (K[63] + st[0]) + (MH_N(63) ? x[63] : (MH_G(63) ? wg[63] : wr[63])));
            } else {
#pragma unroll
                for (int t = 16; t < 64; ++t) sched(t);
#pragma unroll
                for (int t = J + 1; t < 64; ++t)
                    round_kw(A, B, C, D, E, F, G, H,
                             (t >= 16 && MH_R(t)) ? kwr[t] : K[t] + (MH_N(t) ? x[t] : (MH_G(t) ? wg[t] : wr[t])));
                const uint32_t s2[8] = {st[0] + A, st[1] + B, st[2] + C, st[3] + D,
                                        st[4] + E, st[5] + F, st[6] + G, st[7] + H};
                sha256_block_kw_last(s2, a.kw1, h0, a63);  // block 1: padding + length only
                a63 += s2[1] - st[1];                       // so that H1 = st[1] + a63 below
            }
            // New wave best (rare): a uniform branch, so H1 and the
            // lexicographic compare cost nothing on the common path.
            const uint64_t cm = __builtin_amdgcn_ballot_w64(h0 <= wbh0) & valid_mask;
            if (__builtin_expect(cm != 0ull, 0)) {
                const uint32_t h1 = st[1] + a63;
                const uint32_t q = g * 10u + i;
                uint64_t m = cm;
                do {
                    const uint32_t l = (uint32_t)__builtin_ctzll(m);
                    m &= m - 1ull;
                    const uint32_t c0 = (uint32_t)__builtin_amdgcn_readlane((int)h0, (int)l);
                    const uint32_t c1 = (uint32_t)__builtin_amdgcn_readlane((int)h1, (int)l);
                    const uint64_t cn = (wave_u0 + l) * a.pow10L + q;
                    if (c0 < wbh0 || (c0 == wbh0 && (c1 < wbh1 || (c1 == wbh1 && cn < wbn)))) {
                        wbh0 = c0;
                        wbh1 = c1;
                        wbn = cn;
                    }
                } while (m);
            }
        }
    }
#undef MH_N
#undef MH_G
#undef MH_R

    uint64_t hash = ((uint64_t)wbh0 << 32) | wbh1;  // wave-uniform: the wave step of block_min
    uint64_t nonce = wbn;                            // is a no-op, the LDS step joins the waves
    block_min(hash, nonce);
    if (threadIdx.x == 0) partials[blockIdx.x] = Partial{hash, nonce};
}

__global__ __launch_bounds__(kBlockThreads) void generic_scan(const GenArgs a, Partial* __restrict__ partials) {
    using namespace dev;
    const uint32_t gid = blockIdx.x * kBlockThreads + threadIdx.x;
    const uint64_t n = a.first + gid;
    uint32_t h0, h1;
    hash_generic(a, n, h0, h1);
    uint64_t hash = ((uint64_t)h0 << 32) | h1, nonce = n;
    if (gid >= a.count) {
        hash = ~0ull;
        nonce = ~0ull;
    }
    block_min(hash, nonce);
    if (threadIdx.x == 0) partials[blockIdx.x] = Partial{hash, nonce};
}

__global__ __launch_bounds__(kBlockThreads) void hash_batch(const GenArgs a, const uint64_t* __restrict__ nonces,
                                                            uint64_t* __restrict__ out, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlockThreads + threadIdx.x;
    if (i >= n) return;
    uint32_t h0, h1;
    dev::hash_generic(a, nonces[i], h0, h1);
    out[i] = ((uint64_t)h0 << 32) | h1;
}

// One workgroup of 1024 threads; each thread keeps 8 independent 16-byte
// loads in flight, so folding a full 65,536-slot buffer (1 MiB) takes ~8
// load round trips instead of 256 (the loop was latency-bound at 256 threads
// and one load per iteration).
constexpr int kMergeThreads = 1024;
constexpr int kMergeUnroll = 8;

__global__ __launch_bounds__(kMergeThreads) void merge_partials(const Partial* __restrict__ p, uint32_t n,
                                                                Partial* __restrict__ best) {
    using namespace dev;
    uint64_t h = ~0ull, nn = ~0ull;
    for (uint32_t base = 0; base < n; base += kMergeThreads * kMergeUnroll) {
        Partial x[kMergeUnroll];
#pragma unroll
        for (int u = 0; u < kMergeUnroll; ++u) {
            const uint32_t i = base + (uint32_t)u * kMergeThreads + threadIdx.x;
            x[u] = (i < n) ? p[i] : Partial{~0ull, ~0ull};
        }
#pragma unroll
        for (int u = 0; u < kMergeUnroll; ++u)
            if (lex_less(x[u].hash, x[u].nonce, h, nn)) {
                h = x[u].hash;
                nn = x[u].nonce;
            }
    }
    block_min<kMergeThreads>(h, nn);
    if (threadIdx.x == 0) {
        const Partial b = *best;
        if (lex_less(h, nn, b.hash, b.nonce)) *best = Partial{h, nn};
    }
}

// ---------------------------------------------------------------------------
// host-side launchers
// ---------------------------------------------------------------------------
template <int J, int MODE>
static hipError_t launch_fast_t(const FastArgs& a, Partial* partials, uint32_t blocks, hipStream_t s) {
    // MINEHIP_DEV_LDS (experiments only): reserve dynamic LDS per workgroup to
    // cap occupancy, e.g. 54000 -> 3 workgroups (waves/SIMD) per CU.
    static const unsigned lds = [] {
        const char* e = getenv("MINEHIP_DEV_LDS");
        return e ? (unsigned)atoi(e) : 0u;
    }();
    hipLaunchKernelGGL((fast_search<J, MODE>), dim3(blocks), dim3(kBlockThreads), lds, s, a, partials);
    return hipGetLastError();
}

#define MH_CASE(j, m) \
    case j:           \
        return launch_fast_t<j, m>(a, partials, blocks, s);

// MINEHIP_DEV_CODE_OBJECT (experiments only, tools/isa_variant.py): launch
// fast_search<J, MODE> from this gfx950 code object instead of the built-in
// one -- the same kernel with hand-edited ISA, A/B'd in one process.  Read
// on every launch so tools/kbench.py can interleave variants.
static hipError_t launch_fast_dev(const char* path, int J, int mode, const FastArgs& a, Partial* partials,
                                  uint32_t blocks, hipStream_t s) {
    static std::mutex mu;
    static std::map<std::string, hipModule_t> mods;
    hipModule_t mod;
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = mods.find(path);
        if (it == mods.end()) {
            hipError_t e = hipModuleLoad(&mod, path);
            if (e != hipSuccess) return e;
            it = mods.emplace(path, mod).first;
        }
        mod = it->second;
    }
    char name[96];
    snprintf(name, sizeof name, "_ZN2mh11fast_searchILi%dELi%dEEEvNS_8FastArgsEPNS_7PartialE", J, mode);
    hipFunction_t f;
    hipError_t e = hipModuleGetFunction(&f, mod, name);
    if (e != hipSuccess) return e;
    FastArgs args = a;
    Partial* out = partials;
    void* params[] = {&args, &out};
    return hipModuleLaunchKernel(f, blocks, 1, 1, kBlockThreads, 1, 1, 0, s, params, nullptr);
}

hipError_t launch_fast(int J, int mode, const FastArgs& a, Partial* partials, uint32_t blocks, hipStream_t s) {
    if (const char* co = getenv("MINEHIP_DEV_CODE_OBJECT"); co && *co)
        return launch_fast_dev(co, J, mode, a, partials, blocks, s);
    if (mode == kModeOne) {
        switch (J) {
            MH_CASE(0, kModeOne) MH_CASE(1, kModeOne) MH_CASE(2, kModeOne) MH_CASE(3, kModeOne)
            MH_CASE(4, kModeOne) MH_CASE(5, kModeOne) MH_CASE(6, kModeOne) MH_CASE(7, kModeOne)
            MH_CASE(8, kModeOne) MH_CASE(9, kModeOne) MH_CASE(10, kModeOne) MH_CASE(11, kModeOne)
            MH_CASE(12, kModeOne) MH_CASE(13, kModeOne)
            default: return hipErrorInvalidValue;
        }
    }
    if (mode == kModePre) {
        switch (J) {  // last digit at tail byte 64..82 (t <= 63, d <= 20): J <= 4
            MH_CASE(0, kModePre) MH_CASE(1, kModePre) MH_CASE(2, kModePre) MH_CASE(3, kModePre)
            MH_CASE(4, kModePre)
            default: return hipErrorInvalidValue;
        }
    }
    if (mode == kModeTwo) {
        switch (J) {
            MH_CASE(13, kModeTwo) MH_CASE(14, kModeTwo) MH_CASE(15, kModeTwo)
            default: return hipErrorInvalidValue;
        }
    }
    return hipErrorInvalidValue;
}

hipError_t launch_generic_scan(const GenArgs& a, Partial* partials, uint32_t blocks, hipStream_t s) {
    hipLaunchKernelGGL(generic_scan, dim3(blocks), dim3(kBlockThreads), 0, s, a, partials);
    return hipGetLastError();
}

hipError_t launch_hash_batch(const GenArgs& a, const uint64_t* d_nonces, uint64_t* d_out, uint64_t n,
                             hipStream_t s) {
    const uint64_t blocks = (n + kBlockThreads - 1) / kBlockThreads;
    hipLaunchKernelGGL(hash_batch, dim3((uint32_t)blocks), dim3(kBlockThreads), 0, s, a, d_nonces, d_out, n);
    return hipGetLastError();
}

hipError_t launch_merge(const Partial* partials, uint32_t n, Partial* best, hipStream_t s) {
    hipLaunchKernelGGL(merge_partials, dim3(1), dim3(kMergeThreads), 0, s, partials, n, best);
    return hipGetLastError();
}
#undef MH_CASE

}  // namespace mh
