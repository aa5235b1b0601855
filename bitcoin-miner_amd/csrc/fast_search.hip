// fast_search.hip -- the run kernel of libminehip, fast_search<J, MODE>.
//
// Hot path replaced: the miner's scan over bitcoin.Hash (reference
// bitcoin/hash.go:13-17, scan spec SURVEY.md §8(a) A2 / stub
// bitcoin/miner/miner.go:33).  Design: DESIGN.md §2-§4.
//
// One lane = one run of 10^L consecutive nonces that share their d-L higher
// digits; the L lower digits are enumerated in wave-uniform loops (digit
// arithmetic is SALU); only message word J (the last digit's word) changes per
// nonce, so rounds 0..J-1 and every schedule term that does not depend on W[J]
// are hoisted out of the per-nonce loop.
//
// Build (Makefile): this file is compiled to gfx950 assembly only, run through
// the issue-priority pass (issue_prio.py: s_setprio 3 before every run of
// half-rate VALU ops, 0 before every run of full-rate ones),
// assembled into a code object and embedded in libminehip.so (fast_co.S),
// which loads it per device (search_kernels.hip, fast_module).  It is never
// part of the library's fat binary.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernel_common.hpp"
#include "layout.hpp"
#include "sha256_gfx950.hpp"

// Minimum waves per SIMD each fast_search<J, MODE> is compiled for (its register budget): the
// occupancy the layout reaches as a one-chunk-per-workgroup kernel (VGPRs 59..79 -> 7 or 6 waves,
// the Two layouts 98..110 -> 4).  The work-queue loop around the chunk body would otherwise let
// the allocator take 4..6 more VGPRs and cost a wave per SIMD.  -DMH_MIN_WAVES=n overrides all.
// The Early modes (layout.hpp) of the one-block and Pre layouts take 7 (72 VGPRs, spills outside
// the per-nonce loop only): against their layouts' 6, +0.1% to +1.1% on the three buckets of the
// round-5 A/B (profiles/r05d_kbench_early_waves_*.json); TwoEarly keeps Two's 4 (at 6 or 7 it
// spills 56-120 B).  -DMH_EARLY_WAVES=n overrides the One/Pre Early kernels' budget.
// -DMH_ONEPRE_WAVES=n (A/B builds, tools/co_variants.py) sets every One/Pre kernel's budget.
#ifndef MH_EARLY_WAVES
#define MH_EARLY_WAVES 7
#endif
#ifndef MH_ONEPRE_WAVES
#define MH_ONEPRE_WAVES 0
#endif
constexpr int min_waves(int J, int MODE) {
#ifdef MH_MIN_WAVES
    return MH_MIN_WAVES;
#else
    return (MH_ONEPRE_WAVES && MODE % 3 != 2) ? MH_ONEPRE_WAVES
         : (MODE == 3 || MODE == 4) ? MH_EARLY_WAVES
         : MODE % 3 == 2 ? 4
         : MODE % 3 == 1 ? ((J == 0 || J == 4) ? 6 : 7)
                         : ((J == 7 || J == 8 || J >= 10) ? 6 : 7);
#endif
}

namespace mh {

// ---------------------------------------------------------------------------
// fast_search<J, MODE>
// ---------------------------------------------------------------------------
// Inside a lane only message word J (the last digit's word; Early modes: the
// word the innermost digit ends) changes from one nonce to the next, and word
// J-1 (Early: J+1) changes once per group of 10 nonces.  Every
// schedule word W[t] therefore lives at one of three levels, fixed at compile
// time by J:
//   nonce  depends on W[J]                    -> computed per nonce
//   group  depends on W[J-1] (Early: W[J+1]) but not on W[J] -> once per 10 nonces
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

// spread(x, k, w) = x with w zero decimal digits inserted at digit index k (k >= 20: x itself),
// by divisions by the constant 10 (no general 64-bit division); on the rare new-best branch of
// the Early modes only
__device__ __forceinline__ uint64_t spread(uint64_t x, uint32_t k, uint32_t w) {
    if (k >= 20u) return x;
    uint64_t lo = 0, p = 1;
    for (uint32_t j = 0; j < k; ++j) {
        const uint64_t q = x / 10u;
        lo += (x - q * 10u) * p;
        p *= 10u;
        x = q;
    }
    for (uint32_t j = 0; j < w; ++j) p *= 10u;
    return x * p + lo;
}

// One workgroup-sized chunk: the 256 runs u_start + 256 * blk + threadIdx.x, their minimum
// written to partials[blk].
// MODE % 3 is the tail layout (One, Pre, Two); MODE >= 3 (Early): the per-nonce digit ends word
// J and the group digits sit right before it in word J, so no word but J changes inside a run:
// rounds 0..J-1 and every schedule word that does not depend on W[J] are run-level; otherwise
// the per-nonce digit is the last one (word J) and the group digits lie in words J - 1 and J.
template <int J, int MODE>
__device__ __forceinline__ void fast_chunk(const FastArgs& a, Partial* __restrict__ partials, const uint32_t blk) {
    using namespace dev;
    constexpr uint32_t K[64] = MH_K256;
    constexpr int BM = MODE % 3;                          // tail layout
    constexpr bool EARLY = MODE >= 3;
    constexpr int JG = EARLY ? J : J - 1;                 // the other word of the group digits
    constexpr uint64_t NM = Dep::from(J);                 // nonce-level words
    constexpr uint64_t GM = Dep::from(JG) & ~NM;          // group-level words (Early: none)
    constexpr int BASE = (BM == kModePre) ? 16 : 0;       // per-nonce block inside the tail
#define MH_N(t) ((NM >> (t)) & 1ull)
#define MH_G(t) ((GM >> (t)) & 1ull)
#define MH_R(t) (!MH_N(t) && !MH_G(t))
    const uint32_t gid = blk * kBlockThreads + threadIdx.x;
    const uint64_t U = a.u_start + gid;

    // ---- per run --------------------------------------------------------
    // Tail words: host template + the d-L digits of U, right-aligned so U's
    // last digit sits at tail byte hi_end-1 (Early: skipping the L enumerated
    // digits' bytes).  Only words up to the last digit's can receive them
    // (words <= BASE + J, Early BASE + J + 1).
    constexpr int JM = EARLY ? J + 1 : J;                 // the last per-lane word
    constexpr int NW = BASE + JM + 1;
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
                uint32_t pos = a.hi_end - 1u - (uint32_t)k;
                if constexpr (EARLY) pos -= ((uint32_t)k >= a.hole) ? a.hole_w : 0u;
                add_word(w, pos >> 2, dg << (24u - 8u * (pos & 3u)));
            }
        }
    }
    // words of the per-nonce block: per-lane up to JM, uniform (SGPR) after it
    uint32_t W[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) W[t] = (t <= JM) ? w[BASE + t] : a.blk[BASE + t];

    uint32_t st[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) st[i] = a.mid[i];
    if constexpr (BM == kModePre) {
        uint32_t b0[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) b0[t] = w[t];
        sha256_block(st, b0);  // tail block 0 holds no lower digit: once per run
    }
    // rounds 0..J-2 (Early: 0..J-1) read only run-level words
    uint32_t ra = st[0], rb = st[1], rc = st[2], rd = st[3], re = st[4], rf = st[5], rg = st[6], rh = st[7];
#pragma unroll
    for (int t = 0; t < (EARLY ? J : J - 1); ++t) round_kw(ra, rb, rc, rd, re, rf, rg, rh, K[t] + W[t]);

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

    // byte of the per-nonce digit, in word J: the last digit, or (Early) the innermost one
    const uint32_t lastpos = EARLY ? a.inner : a.lo_pos + a.L - 1u;
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
    const uint64_t wave_u0 = a.u_start + (uint64_t)blk * kBlockThreads + wave * 64u;
    uint32_t wbh0 = 0xFFFFFFFFu, wbh1 = 0xFFFFFFFFu;
    uint64_t wbn = ~0ull;

    for (uint32_t g = 0; g < a.n_groups; ++g) {
        // ---- per group of 10 nonces --------------------------------------
        // the L-1 digits of g: wave-uniform, so this is SALU work.  Into word J (cj) or word
        // J - 1 (cjm; the Early layouts put every group digit in word J)
        uint32_t cj = 0u, cjm = 0u, gq = g;
        if constexpr (!EARLY) {
            // digits 0..L-2 of q = 10*g + i, at bytes lo_pos .. lo_pos+L-2
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
        } else {
            // g's digit j (least significant first) at byte g_last - j, one more to the left
            // from j = g_hole on (the innermost digit's decimal place); every one in word J
            // (make_fast_args builds only such pieces, enqueue_piece re-checks each one)
            for (uint32_t j = 0; j + 1u < a.L; ++j) {
                const uint32_t q = gq / 10u;
                const uint32_t dg = gq - q * 10u;
                gq = q;
                const uint32_t p = a.g_last - j - (j >= a.g_hole ? 1u : 0u);
                cj += dg << (24u - 8u * (p & 3u));
            }
        }
        const uint32_t wJ = W[J] + cj;  // word J with this group's digits, the per-nonce digit '0'
        const uint32_t s0wJ = ssig0(wJ), s1wJ = ssig1(wJ);
        uint32_t wg[64], pg[64];
        if constexpr (!EARLY && J > 0) wg[J - 1] = W[J - 1] + cjm;
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
        // round J-1 reads the group-level word J-1 (Early: it is run-level, done above)
        uint32_t ga = ra, gb = rb, gc = rc, gd = rd, ge = re, gf = rf, gG = rg, gh = rh;
        if constexpr (!EARLY && J > 0) round_kw(ga, gb, gc, gd, ge, gf, gG, gh, K[J - 1] + wg[J - 1]);
        // round J: every input but W[J]'s last digit is known here
        const uint32_t t1J = (gh + (K[J] + wJ)) + bsig1(ge) + ch(ge, gf, gG);
        const uint32_t t2J = bsig0(ga) + maj(ga, gb, gc);

        for (uint32_t i = 0; i < 10u; ++i) {
            // ---- per nonce ------------------------------------------------
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
            if constexpr (BM != kModeTwo) {
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
            uint64_t cm = __builtin_amdgcn_ballot_w64(h0 <= wbh0) & valid_mask;
            if (__builtin_expect(cm != 0ull, 0)) {
                const uint32_t h1 = st[1] + a63;
                const uint32_t q = g * 10u + i;
                // Many candidates (the first nonce of a run makes every lane one): keep only
                // the lanes holding their smallest H0, found by a DPP wave-min, instead of a
                // 64-step scalar scan (~1,000 serial SALU / readlane instructions per run).
                if (__builtin_popcountll(cm) > 4) {
                    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
                    const uint32_t mh = wave_min_u32(((cm >> lane) & 1ull) ? h0 : 0xFFFFFFFFu);
                    cm &= __builtin_amdgcn_ballot_w64(h0 == mh);
                }
                uint64_t m = cm;
                do {
                    const uint32_t l = (uint32_t)__builtin_ctzll(m);
                    m &= m - 1ull;
                    const uint32_t c0 = (uint32_t)__builtin_amdgcn_readlane((int)h0, (int)l);
                    const uint32_t c1 = (uint32_t)__builtin_amdgcn_readlane((int)h1, (int)l);
                    uint64_t cn;
                    if constexpr (!EARLY)
                        cn = (wave_u0 + l) * a.pow10L + q;
                    else
                        cn = spread(wave_u0 + l, a.hole, a.hole_w) * a.u_mul + spread(g, a.g_hole, 1u) * a.g_mul +
                             i * a.i_mul;
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
    if (threadIdx.x == 0) partials[blk] = Partial{hash, nonce};
}

// The chunk the workgroup runs next: thread 0 takes it from the launch's counter (a vector
// atomic, returning the old value), LDS hands it to the other waves.
__device__ __forceinline__ uint32_t claim_chunk(uint32_t* counter) {
    __shared__ uint32_t s_next;
    if (threadIdx.x == 0) s_next = atomicAdd(counter, 1u);
    __syncthreads();
    const uint32_t blk = __builtin_amdgcn_readfirstlane(s_next);  // one value per workgroup: scalar
    __syncthreads();  // every wave has read it before thread 0 may overwrite it
    return blk;
}

template <int J, int MODE>
__global__ __launch_bounds__(kBlockThreads, min_waves(J, MODE)) void fast_search(const FastArgs a,
                                                                           Partial* __restrict__ partials) {
    // Static: workgroup b runs chunk b.  Work queue (a.counter set, grid <= the resident
    // workgroups): each workgroup claims chunks until the counter passes n_chunks; every
    // workgroup leaves once a claim comes back >= n_chunks, so the grid always drains.
    // The chunk body reads its arguments through a pointer the loop launders every iteration,
    // so the compiler cannot keep values derived from them live from one chunk to the next:
    // hoisted out of the loop they spilled ~240 SGPRs into VGPR lanes (85 VGPRs instead of 70).
    using KArgs = __attribute__((address_space(4))) const FastArgs;
    KArgs* const kp = (KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    uint32_t blk = a.counter ? claim_chunk(a.counter) : blockIdx.x;
    while (blk < a.n_chunks) {
        KArgs* k = kp;
        asm volatile("" : "+s"(k));
        fast_chunk<J, MODE>(*(const FastArgs*)k, partials, blk);
        if (!a.counter) break;
        blk = claim_chunk(a.counter);
    }
}

// Marker of a code object whose fast_search kernels run the work-queue loop above over this
// FastArgs layout: its size is sizeof(FastArgs).  The library uses the work queue with a code
// object only if it carries the marker at that size (search_kernels.hip, fast_function) -- the
// embedded object always does; one loaded by the dev build's MINEHIP_DEV_CODE_OBJECT hook from
// older sources runs one workgroup per chunk instead of searching only its first chunks.
extern "C" {
__device__ __attribute__((used)) uint8_t mh_fast_queue_args[sizeof(FastArgs)];
}

// The instantiations the planner uses (plan.cpp; launch by mangled name in
// search_kernels.hip): kModeOne for every word J of the last digit in a
// one-block tail, kModePre for J <= 4 of block 1 (last digit at tail byte
// 64..82), kModeTwo for J = 13..15 of block 0; the Early modes where a nonce
// costs less with the digit ending word J innermost than with the last digit
// in word J + 1 (plan.cpp: nonce_cost(J) < nonce_cost(J + 1)).
#define MH_INST(j, m) template __global__ void fast_search<j, m>(const FastArgs, Partial* __restrict__);
MH_FAST_KERNELS(MH_INST)  // layout.hpp: the one list of instantiated layouts
#undef MH_INST

}  // namespace mh
