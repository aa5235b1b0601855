// plan.hpp -- host-side search planning for libminehip (no HIP dependency).
//
// Splits a Request range [lower, upper] (bitcoin/message.go:18-34) into
// kernel launches: per decimal-length bucket, the nonces that form whole runs
// of 10^L go to fast_search, the ragged edges and tiny buckets go to
// generic_scan.  The prefix "msg " is absorbed here into a SHA-256 midstate
// (the constant part of fmt.Sprintf("%s %d") at bitcoin/hash.go:15).
#pragma once
#include <stdint.h>
#include <stddef.h>

#include <functional>
#include <vector>

#include "layout.hpp"

namespace mh {

// Every full 64-byte block of P = msg ' ' compressed into mid; the rest of P
// is the tail.
struct Prefix {
    uint32_t mid[8];
    uint8_t tail[64];
    uint32_t t;     // len(P) mod 64
    uint64_t plen;  // len(P) = len(msg) + 1
};

void absorb_prefix(const uint8_t* msg, size_t len, Prefix* out);

// FIPS 180-4 compression on the host (midstates and the fixed schedule of a
// padding-only block).
void host_compress(uint32_t st[8], const uint32_t w16[16]);

// One launch of the plan.
struct Piece {
    uint64_t first;   // first nonce
    uint64_t count;   // nonces
    int kind;         // 0 fast, 1 generic
    int digits;
    int L;            // fast only
    int J;            // fast only
    int mode;         // fast only: FastMode
    int blocks;       // tail blocks of the final message
    uint32_t ops;     // fast only: nonce_cost(J, mode).ops
    uint32_t slots;   // fast only: nonce_cost(J, mode).slots
    FastArgs fa;      // kind 0
    GenArgs ga;       // both (generic launch args; also used by hash_batch)
};

struct PlanOpts {
    // L <= 3 (round 2: then with >= 2^21 runs per bucket) and up to 2^34 nonces (~67k
    // workgroups at L = 3) per launch.  With the issue-priority build the per-run work
    // (digit formatting, hoisted rounds, the first-nonce candidate scan, wave
    // start and the workgroup reduction) costs more than the longer tail of
    // 1,000-nonce lanes: +2% on configs[1], +5% / +4% on configs[2]'s halves,
    // +3% on configs[3] against L <= 2, 2^23 runs, 2^32-nonce launches, the
    // round-1 choice (profiles/r02ap_kbench_plan.json).
    int lower_digits = 3;                        // L upper bound (nonces per lane = 10^L)
    // Lower L until a bucket has min_lanes runs: 2^19 runs = 2,048 workgroups, about one generation
    // of the resident grid (7 x 256 CUs).  Round 4, with work queues and two streams, A/B in one
    // process against the round-2 2^21: configs[1] +1.4% (its d = 9 bucket now runs 1,000-nonce
    // lanes), configs[2] +0.4% / +0.6%; 2^16 (buckets of a fifth of a generation at L = 3) -4.7%
    // (profiles/r04c_kbench_min_lanes_*.json).
    uint64_t min_lanes = 1u << 19;
    // Nonces per fast launch: 2^35, so with the 2^17-workgroup cap one launch takes up to ~3.4e10
    // nonces at L = 3 (~0.6 s with one tail block).  A bucket's launches run back to back on the
    // high-priority stream and every boundary drains; round 4 against 2^34, A/B in one process: a
    // configs[3] step (5.5e10 nonces, 2 launches instead of 4) +0.52% / +0.58% on two boxes, a
    // 2-GPU shard +0.41%, configs[1] and [2] unchanged plans (profiles/r04r_kbench_launch_size_*.json).
    uint64_t max_nonces_per_launch = 1ull << 35;
    uint32_t max_blocks = 1u << 17;              // workgroups per launch (<= kMaxBlocksPerLaunch; +0.1% over 2^16)
    uint64_t generic_below = 1u << 20;           // a bucket this small goes to the generic kernel whole
    // Execution (minehip.cpp, not the plan itself): 1 = every piece on one stream in nonce
    // order; 2 = the pieces at the full L (coarse: 1,000-nonce lanes) on a high-priority
    // stream, the others (shorter lanes, generic edges) on a low-priority one, so that the
    // short workgroups back-fill the coarse launch's tail instead of each launch draining alone.
    // Tail split: the last fine_tail nonces (whole runs) of every bucket planned at the full L
    // go out as one more piece at L - 1 -- 100-nonce lanes whose workgroups end ~10x sooner --
    // so that the coarse launch's drain has short work to back-fill.  0: off.
    // Round 3 (profiles/r03d_*): 2 streams + a 2^28-nonce tail against one stream,
    // wall clock, A/B in one process: configs[1] +1.6%, configs[2] +1.0% / +1.1%, an 8-GPU
    // configs[3] shard +0.2%, and the predicted 8-GPU per-GPU efficiency 0.982 -> 1.00.
    int streams = 2;
    uint64_t fine_tail = 1ull << 28;
    // Work queue (execution): a fast launch's workgroups claim 256-run chunks from a counter
    // instead of one chunk each, so the 8 XCDs, whose clocks differ by a few percent, finish
    // together.  Round 3, A/B in one process against one chunk per workgroup
    // with the same code object: +0.6% to +1.9% on configs[1], configs[2]'s halves and the d = 10
    // bucket (profiles/r03u_*).  0: one workgroup per chunk.
    int queue = 1;
    // Innermost digit (execution of the plan's fast pieces): 1 = where a nonce costs
    // less with the digit ending the word before the last digit's enumerated innermost (the
    // kMode*Early layouts, layout.hpp), take that layout; 0 = always the last digit.
    int early = 1;
    // Round 4 A/B-rejected three more execution knobs and they were removed from the library in
    // round 5 (HISTORY.md §3): full-L pieces below 2^31 / 2^33 nonces on the low-priority stream
    // (-4% / -5%), a finest tail at L - 2 on a third stream (+-0.3%), and the tail split fused
    // into the coarse launch's work queue (-0.2% to -1.0%).
};

// Calls cb for every piece in increasing nonce order; stops early when cb
// returns false.  lower <= upper required.  A fast piece lies in one decimal
// bucket; a generic piece may span several (contiguous small buckets and
// edges are coalesced into one launch).
void plan_search(const Prefix& pre, uint64_t lower, uint64_t upper, const PlanOpts& opt,
                 const std::function<bool(const Piece&)>& cb);

// Generic-kernel arguments for this prefix (first/count left 0).
void make_gen_args(const Prefix& pre, GenArgs* ga);

// Algorithmic VALU instructions per nonce of a fast piece: the SHA-256 work
// that depends on the nonce's last digit (word J), with gfx950's 3-input ops
// (14 per round, 4 per sigma, add3 sums); work shared by a group or a run is
// amortised like the host midstate of SURVEY.md §8(d).  DESIGN.md §4.
uint32_t nonce_ops(int J, int mode);

// The same work in SIMD-32 issue slots (full-rate op 1, v_alignbit 2, one per
// addition) -- the unit of the roofline peak, 128 lanes/clk/CU.
struct NonceCost {
    uint32_t ops, slots;
};
NonceCost nonce_cost(int J, int mode);

int decimal_digits(uint64_t n);

// ---- relative search cost, for splitting a range over devices (mh_search_multi) ----
// One segment per decimal bucket of [lower, upper]: every nonce of [a, b] costs `per` issue slots
// -- the fast kernel's nonce_cost slots at the bucket's planned L (shorter lanes a few percent
// more), or kGenericSlotsPerBlock per tail block for a bucket the planner gives the generic
// kernel.  A device's rate in these units (slots per ns) does not depend on which layouts its
// range happened to hold, so rates measured on one range size the shards of the next.
struct CostSeg {
    uint64_t a, b;  // inclusive
    double per;
    // the bucket runs at the full L in a launch of many generations of workgroups (>= 2^21 runs):
    // its time follows `per`; the shorter-lane, few-generation and generic buckets run a few to
    // ~20% off the model (drains), so a device's rate is only measured on steady spans
    bool steady;
};
// Share of [lo, hi]'s cost in segments that are not steady.
double unsteady_share(const std::vector<CostSeg>& segs, uint64_t lo, uint64_t hi);
constexpr double kGenericSlotsPerBlock = 2.0 * 1760.0;  // estimate: a full compression + per-nonce formatting
constexpr double kUnsteadyFactor = 1.15;                 // fast buckets that are not steady (below)
void cost_segments(const Prefix& pre, uint64_t lower, uint64_t upper, const PlanOpts& opt,
                   std::vector<CostSeg>* out);
double segments_cost(const std::vector<CostSeg>& segs, uint64_t lo, uint64_t hi);

struct Span {
    uint64_t lo, hi;  // inclusive
    bool empty;
};
// Cut the segments' range into w.size() contiguous spans in order, span k carrying a share of the
// total cost proportional to w[k] (>= 0).  The spans tile the range exactly (integer cut
// positions); a span whose share rounds to no nonce is empty.
void split_by_cost(const std::vector<CostSeg>& segs, const std::vector<double>& w, std::vector<Span>* out);

}  // namespace mh
