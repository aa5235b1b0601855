// layout.hpp -- host/device shared launch descriptors for libminehip.
//
// The message the reference hashes per nonce is  msg ' ' decimal(nonce)
// (bitcoin/hash.go:15).  The host absorbs every full 64-byte block of the
// constant prefix P = msg ' ' into a midstate; what remains is the "tail":
// t = len(P) mod 64 prefix bytes, then the d digits, 0x80, zeros and the
// 64-bit bit length -- one or two 64-byte tail blocks (tail byte positions
// 0..127, big-endian words 0..31).
//
// A search over one decimal-length bucket (all nonces have d digits) splits
// every nonce n = U * 10^L + q into a run index U (the d-L "higher" digits,
// one run per GPU lane) and q in [0, 10^L) (the L "lower" digits, enumerated
// inside the lane).  See DESIGN.md §3.
#pragma once
#include <stdint.h>

namespace mh {

constexpr int kBlockThreads = 256;         // 4 waves of 64 per workgroup
constexpr uint32_t kMaxBlocksPerLaunch = 1u << 18;  // partials buffer slots; hard cap of one grid

struct Partial {          // one (hash, nonce) candidate; ordered lexicographically
    uint64_t hash;
    uint64_t nonce;
};

enum FastMode : uint32_t {
    kModeOne = 0,   // one tail block, compressed per nonce from the host midstate
    kModePre = 1,   // two tail blocks; block 0 holds no lower digit and is compressed once per run
    kModeTwo = 2,   // two tail blocks; the lower digits sit in block 0 -> both blocks per nonce
    // The same three tail layouts with an earlier innermost digit (mode - 3 is the tail layout):
    // the digit enumerated per nonce is not the last one but the digit ending word J, the word
    // before the last digit's, at decimal position p = 1..4, and the other enumerated digits (a
    // group, per 10 nonces) are the L - 1 right before it in word J.  A nonce then costs
    // nonce_cost(J) instead of nonce_cost(J + 1), which is less for J + 1 = 1 (W[1] reaches W[16]
    // through sigma0), J + 1 = 9 (W[9] is W[16]'s t-7 term) and J + 1 = 14, and
    // only word J changes inside a lane.  A lane's nonces are not contiguous: its U digits are the
    // p below and the ones above the L enumerated positions p .. p+L-1.
    kModeOneEarly = 3,
    kModePreEarly = 4,
    kModeTwoEarly = 5,
};
constexpr int kModes = 6;

// The instantiated fast_search<J, MODE> kernels: every layout a bucket with d <= 20 can produce
// (One J = 0..13, Pre J = 0..4, Two J = 13..15) and the Early layouts the planner takes (One
// J = 0, 8, Pre J = 0, Two J = 13).  The one list: fast_search.hip instantiates it, the planner
// (plan.cpp) and the launcher (search_kernels.hip) accept exactly it, csrc/loop_mix.py and the
// tests read it from here.
#define MH_FAST_KERNELS(X)                                                                                 \
    X(0, kModeOne) X(1, kModeOne) X(2, kModeOne) X(3, kModeOne) X(4, kModeOne) X(5, kModeOne)              \
    X(6, kModeOne) X(7, kModeOne) X(8, kModeOne) X(9, kModeOne) X(10, kModeOne) X(11, kModeOne)            \
    X(12, kModeOne) X(13, kModeOne)                                                                        \
    X(0, kModePre) X(1, kModePre) X(2, kModePre) X(3, kModePre) X(4, kModePre)                             \
    X(13, kModeTwo) X(14, kModeTwo) X(15, kModeTwo)                                                        \
    X(0, kModeOneEarly) X(8, kModeOneEarly) X(0, kModePreEarly) X(13, kModeTwoEarly)

struct FastKernelId {
    int J;
    int mode;
};
#define MH_FAST_KERNEL_ID(j, m) FastKernelId{j, m},
constexpr FastKernelId kFastKernels[] = {MH_FAST_KERNELS(MH_FAST_KERNEL_ID)};
#undef MH_FAST_KERNEL_ID
constexpr int kNumFastKernels = (int)(sizeof(kFastKernels) / sizeof(kFastKernels[0]));

constexpr bool fast_kernel_exists(int J, int mode) {
    for (const FastKernelId& k : kFastKernels)
        if (k.J == J && k.mode == mode) return true;
    return false;
}
constexpr uint32_t kNoHole = 20;  // a digit index no layout reaches (d <= 20)

// Arguments of the fast (run) kernel.  Passed by value: lands in SGPRs.
struct FastArgs {
    uint32_t mid[8];      // chaining state before tail block 0
    uint32_t blk[32];     // tail words: prefix bytes, '0' at every digit byte, 0x80, bit length
    uint64_t u_start;     // run index U of lane 0 of block 0
    uint64_t pow10L;      // 10^L
    uint32_t n_runs;      // active lanes in this launch
    uint32_t hi_end;      // tail byte index one past U's last digit
    uint32_t n_hi;        // digits of U (= d - L)
    uint32_t lo_pos;      // byte index (within the per-nonce block) of the first lower digit
    uint32_t L;           // lower digits enumerated inside a lane (1..5)
    uint32_t n_groups;    // 10^(L-1): groups of 10 consecutive nonces per lane
    uint32_t mode;        // FastMode
    uint32_t n_chunks;    // workgroup-sized chunks (256 runs each) in this launch
    // Early modes only (the per-run digit formatting and the nonce of a candidate):
    //   U's digit k sits at tail byte hi_end - 1 - k - (k >= hole ? hole_w : 0), the group's
    //   digit j at per-nonce-block byte g_last - j - (j >= g_hole), the innermost digit at byte
    //   `inner`; nonce(U, g, i) = spread(U, hole, hole_w) * u_mul + spread(g, g_hole, 1) * g_mul
    //   + i * i_mul, where spread(x, k, w) inserts w zero decimal digits at digit index k
    //   (k >= 20: x itself).
    uint32_t inner;
    uint32_t hole;
    uint32_t g_last;
    uint32_t g_hole;
    uint32_t hole_w;
    uint32_t pad_;
    uint64_t u_mul;
    uint64_t g_mul;
    uint64_t i_mul;
    uint32_t kw1[64];     // kModeTwo: K[i] + W[i] of tail block 1 (padding + length only)
    // Work queue: non-null -> the launch's workgroups claim chunks from this zeroed device
    // counter until it passes n_chunks, so an XCD that clocks faster takes more of them;
    // null -> workgroup b runs chunk b (grid = n_chunks).  DESIGN.md §3.
    uint32_t* counter;
};

// Arguments of the generic per-nonce kernels (range edges, small buckets,
// batch hashing): any nonce, any digit count, one nonce per lane.
struct GenArgs {
    uint32_t mid[8];      // chaining state before tail block 0
    uint32_t tail[16];    // the t prefix bytes of the tail, zero elsewhere
    uint64_t plen;        // len(msg) + 1 (bytes before the digits, all blocks)
    uint64_t first;       // scan: first nonce
    uint64_t count;       // scan: nonces in this launch
    uint32_t t;           // tail prefix length, 0..63
    uint32_t pad;
};

}  // namespace mh
