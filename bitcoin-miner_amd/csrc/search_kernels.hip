// search_kernels.hip -- gfx950 kernels of libminehip (fat binary) and the
// launchers of every kernel, including the embedded fast_search module.
//
// Hot path replaced: the miner's scan over bitcoin.Hash (reference
// bitcoin/hash.go:13-17, scan spec SURVEY.md §8(a) A2 / stub
// bitcoin/miner/miner.go:33).  Design: DESIGN.md §3.
//
//   fast_search<J, MODE>  (fast_search.hip) the run kernel; it reaches the
//                         library as a code object built through the
//                         issue-priority pass and is launched from here by
//                         name (fast_module below).
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

#include <algorithm>
#include <stdio.h>
#include <stdlib.h>

#include <map>
#include <mutex>
#include <string>
#include <utility>

#include "kernel_common.hpp"
#include "layout.hpp"
#include "sha256_gfx950.hpp"

// fast_search.hip's code object after the issue-priority pass (fast_co.S)
extern "C" const unsigned char mh_fast_co_begin[];

namespace mh {
namespace dev {

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
// fast_search<J, MODE> lives in a code object of its own, loaded once per
// device and launched by its mangled name.  The product library knows only the
// embedded code object.  The dev build (`make dev`, -DMH_DEV_HOOKS,
// build/dev/libminehip.so; never shipped as the package's library) also
// reads MINEHIP_DEV_CODE_OBJECT, a code object file to use instead (e.g. the
// same kernels without the issue-priority pass, tools/isa_variant.py), on
// every launch so that tools/kbench.py can interleave variants in one process.
namespace {
std::mutex g_mod_mu;
std::map<std::pair<std::string, int>, hipModule_t> g_mods;                    // (file or "", dev)
std::map<std::pair<hipModule_t, int>, hipFunction_t> g_funcs;                // (module, J + 16 * mode)
std::map<hipModule_t, bool> g_queue_ok;  // the module's kernels run the work-queue loop (marker)

// queue_ok: the code object carries fast_search.hip's mh_fast_queue_args marker at this
// library's sizeof(FastArgs), i.e. its kernels claim chunks from a.counter
hipError_t fast_function(int dev, int J, int mode, hipFunction_t* f, bool* queue_ok = nullptr) {
#ifdef MH_DEV_HOOKS
    const char* co = getenv("MINEHIP_DEV_CODE_OBJECT");
    const std::string path = (co && *co) ? co : "";
#else
    const std::string path;
#endif
    std::lock_guard<std::mutex> g(g_mod_mu);
    auto it = g_mods.find({path, dev});
    if (it == g_mods.end()) {
        hipModule_t m;
        const hipError_t e = path.empty() ? hipModuleLoadData(&m, mh_fast_co_begin) : hipModuleLoad(&m, path.c_str());
        if (e != hipSuccess) {
            (void)hipGetLastError();  // the failure is returned here; do not leave it for the next launch check
            return e;
        }
        it = g_mods.emplace(std::make_pair(path, dev), m).first;
        hipDeviceptr_t gp = nullptr;
        size_t gsz = 0;
        const bool marked = hipModuleGetGlobal(&gp, &gsz, m, "mh_fast_queue_args") == hipSuccess &&
                            gsz == sizeof(FastArgs);
        (void)hipGetLastError();
        g_queue_ok[m] = marked;
    }
    if (queue_ok) *queue_ok = g_queue_ok[it->second];
    auto fit = g_funcs.find({it->second, J + 16 * mode});
    if (fit == g_funcs.end()) {
        char name[96];
        snprintf(name, sizeof name, "_ZN2mh11fast_searchILi%dELi%dEEEvNS_8FastArgsEPNS_7PartialE", J, mode);
        hipFunction_t fn;
        const hipError_t e = hipModuleGetFunction(&fn, it->second, name);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            return e;
        }
        fit = g_funcs.emplace(std::make_pair(it->second, J + 16 * mode), fn).first;
    }
    *f = fit->second;
    return hipSuccess;
}

bool fast_variant_exists(int J, int mode) { return fast_kernel_exists(J, mode); }  // layout.hpp MH_FAST_KERNELS
}  // namespace

// Load the fast_search module on dev (the current device) at context setup,
// so the first search does not pay for it.
hipError_t fast_module_init(int dev) {
    hipFunction_t f;
    return fast_function(dev, 4, kModeOne, &f);
}

// Workgroups of f that fit on dev at once (occupancy x CUs), cached per function.
hipError_t resident_groups(int dev, hipFunction_t f, unsigned lds, uint32_t* out) {
    static std::mutex mu;
    static std::map<std::pair<hipFunction_t, unsigned>, uint32_t> cache;
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find({f, lds});
    if (it == cache.end()) {
        int per_cu = 0, cus = 0;
        hipError_t e = hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, kBlockThreads, lds);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            return e;
        }
        it = cache.emplace(std::make_pair(f, lds), (uint32_t)std::max(1, per_cu) * (uint32_t)std::max(1, cus)).first;
    }
    *out = it->second;
    return hipSuccess;
}

// a.n_chunks chunks of 256 runs; static (a.counter null): one workgroup per chunk; work queue:
// as many workgroups as fit at once (an over-estimate only queues some of them), each claiming
// chunks from a.counter (zeroed by the caller, one counter per launch).
hipError_t launch_fast(int dev, int J, int mode, const FastArgs& a, Partial* partials, hipStream_t s) {
    if (!fast_variant_exists(J, mode)) return hipErrorInvalidValue;
#ifdef MH_DEV_HOOKS
    // MINEHIP_DEV_LDS (dev build only): reserve dynamic LDS per workgroup to
    // cap occupancy, e.g. 54000 -> 3 workgroups (waves/SIMD) per CU.  Read at every launch, so
    // that one A/B process can interleave settings.
    const char* lds_env = getenv("MINEHIP_DEV_LDS");
    const unsigned lds = lds_env ? (unsigned)atoi(lds_env) : 0u;
#else
    constexpr unsigned lds = 0;
#endif
    hipFunction_t f;
    bool queue_ok = false;
    hipError_t e = fast_function(dev, J, mode, &f, &queue_ok);
    if (e != hipSuccess) return e;
    FastArgs args = a;
    if (!queue_ok) args.counter = nullptr;  // a code object without the loop: one workgroup per chunk
    uint32_t grid = args.n_chunks;
    if (args.counter) {
        uint32_t resident = 0;
        e = resident_groups(dev, f, lds, &resident);
        if (e != hipSuccess) return e;
        grid = std::min(grid, resident);
    }
    Partial* out = partials;
    void* params[] = {&args, &out};
    return hipModuleLaunchKernel(f, grid, 1, 1, kBlockThreads, 1, 1, lds, s, params, nullptr);
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

}  // namespace mh
