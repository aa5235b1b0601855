// salu_coissue.hip -- does scalar-unit (SALU) SHA-256 work co-issue for free
// next to a VALU-bound SHA-256 stream on gfx950?  (DESIGN.md §9 experiment.)
//
// One kernel, two roles picked per workgroup (uniform branch):
//   VALU role   every lane runs sha256_block (the product's VALU compression,
//               14 ops/round) VITERS times on lane-varying data;
//   SALU role   every wave runs compressions on wave-uniform data in SGPRs
//               (s_lshr_b64 on {x, x} for rotations, s_xor/s_and/s_add for
//               the rest) until the first VALU wave has finished.
// Workgroups with blockIdx % P == P-1 take the SALU role (P = 0: none), so
// the VALU workgroups are the same in every configuration.  Each wave stores
// its s_memtime duration and work; comparing the VALU waves' cycles with and without
// SALU neighbours answers whether the scalar hashes are free.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o build/salu_coissue tools/salu_coissue.hip
// Output: one JSON line.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../bitcoin-miner_amd/csrc/sha256_gfx950.hpp"

using namespace mh::dev;

template <int N>
__device__ __forceinline__ uint32_t srotr(uint32_t x) {
    const uint64_t p = ((uint64_t)x << 32) | x;
    uint64_t r;
    asm("s_lshr_b64 %0, %1, %2" : "=s"(r) : "s"(p), "n"(N));
    return (uint32_t)r;
}
__device__ __forceinline__ uint32_t s_bsig0(uint32_t a) { return srotr<2>(a) ^ srotr<13>(a) ^ srotr<22>(a); }
__device__ __forceinline__ uint32_t s_bsig1(uint32_t e) { return srotr<6>(e) ^ srotr<11>(e) ^ srotr<25>(e); }
__device__ __forceinline__ uint32_t s_ssig0(uint32_t x) { return srotr<7>(x) ^ srotr<18>(x) ^ (x >> 3); }
__device__ __forceinline__ uint32_t s_ssig1(uint32_t x) { return srotr<17>(x) ^ srotr<19>(x) ^ (x >> 10); }

// Scalar compression with a rolling 16-word schedule window (SGPR budget).
__device__ __forceinline__ void s_compress(uint32_t st[8], uint32_t w[16]) {
    constexpr uint32_t K[64] = MH_K256;
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            wi = w[i & 15] + w[(i - 7) & 15] + s_ssig0(w[(i - 15) & 15]) + s_ssig1(w[(i - 2) & 15]);
            w[i & 15] = wi;
        }
        const uint32_t t1 = h + s_bsig1(e) + ((e & f) ^ (~e & g)) + K[i] + wi;
        const uint32_t t2 = s_bsig0(a) + ((a & b) ^ (c & (a ^ b)));
        h = g; g = f; f = e; e = d + t1;
        d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

__global__ __launch_bounds__(256) void coissue(int P, int viters, uint32_t seed, uint64_t* cyc, uint32_t* out,
                                               int* stop) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool salu = P > 0 && (int)(blockIdx.x % (unsigned)P) == P - 1;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    uint32_t acc, done = 0;
    if (salu) {
        // until the first VALU wave finishes (then at most one more compression)
        uint32_t st[8], w[16];
        const uint32_t s = __builtin_amdgcn_readfirstlane(seed ^ (blockIdx.x * 4u + (uint32_t)wave));
#pragma unroll
        for (int i = 0; i < 8; ++i) st[i] = s * (2u * i + 1u);
        do {
#pragma unroll
            for (int i = 0; i < 16; ++i) w[i] = st[i & 7] ^ (done + (uint32_t)i);
            s_compress(st, w);
            ++done;
        } while (__hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0);
        acc = st[0] ^ st[1];
    } else {
        uint32_t st[8], w[16];
        const uint32_t s = seed ^ (blockIdx.x * 256u + threadIdx.x);
#pragma unroll
        for (int i = 0; i < 8; ++i) st[i] = s * (2u * i + 1u);
        for (int it = 0; it < viters; ++it) {
#pragma unroll
            for (int i = 0; i < 16; ++i) w[i] = st[i & 7] ^ (uint32_t)(it + i);
            sha256_block(st, w);
        }
        acc = st[0] ^ st[1];
        done = (uint32_t)viters;
        if (lane == 0) __hip_atomic_store(stop, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        cyc[2 * (blockIdx.x * 4 + wave)] = (t1 - t0) | ((uint64_t)salu << 63);
        cyc[2 * (blockIdx.x * 4 + wave) + 1] = done;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;  // keep live
}

// Every workgroup is resident at once (5 per CU at <= 96 VGPRs), so each
// run is one steady state: A = 4 VALU waves/SIMD, B = the same + 1 SALU wave
// per SIMD, C = 5 VALU waves/SIMD.
int main(int argc, char** argv) {
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    const int viters = argc > 1 ? atoi(argv[1]) : 256;
    const size_t maxb = (size_t)cus * 5;
    uint64_t* cyc;
    uint32_t* out;
    int* stop;
    (void)hipMalloc(&cyc, maxb * 4 * 16);
    (void)hipMalloc(&out, maxb * 4);
    (void)hipMalloc(&stop, 4);
    hipEvent_t ea, eb;
    (void)hipEventCreate(&ea);
    (void)hipEventCreate(&eb);
    printf("{\"cus\": %d, \"viters\": %d, \"runs\": [", cus, viters);
    struct Cfg { const char* name; int P, wgs_per_cu; } cfgs[] = {
        {"A_4valu", 0, 4}, {"B_4valu_1salu", 5, 5}, {"C_5valu", 0, 5}, {"A_4valu", 0, 4}, {"B_4valu_1salu", 5, 5}};
    for (int ci = 0; ci < 5; ++ci) {
        const Cfg& c = cfgs[ci];
        const int blocks = cus * c.wgs_per_cu;
        for (int rep = 0; rep < 2; ++rep) {  // rep 0 warms up
            (void)hipMemset(stop, 0, 4);
            (void)hipEventRecord(ea);
            coissue<<<blocks, 256>>>(c.P, viters, 7u + rep, cyc, out, stop);
            (void)hipEventRecord(eb);
            (void)hipEventSynchronize(eb);
        }
        float ms;
        (void)hipEventElapsedTime(&ms, ea, eb);
        uint64_t* h = (uint64_t*)malloc((size_t)blocks * 4 * 16);
        (void)hipMemcpy(h, cyc, (size_t)blocks * 4 * 16, hipMemcpyDeviceToHost);
        double vc = 0, sc = 0, sdone = 0, vdone = 0;
        long nv = 0, ns = 0;
        for (long i = 0; i < (long)blocks * 4; ++i) {
            const double cy = (double)(h[2 * i] & ~(1ull << 63));
            if (h[2 * i] >> 63) { sc += cy; sdone += (double)h[2 * i + 1]; ++ns; }
            else { vc += cy; vdone += (double)h[2 * i + 1]; ++nv; }
        }
        free(h);
        // per SIMD: VALU lane-compressions and SALU compressions per 1000 cycles
        const double simds = cus * 4.0;
        const double vrate = nv ? (vdone * 64.0 / simds) / (vc / nv) * 1000.0 : 0.0;
        const double srate = ns ? (sdone / simds) / (sc / ns) * 1000.0 : 0.0;
        printf("%s{\"cfg\": \"%s\", \"blocks\": %d, \"ms\": %.3f, \"valu_wave_cycles\": %.0f, "
               "\"salu_wave_cycles\": %.0f, \"salu_comp_per_wave\": %.1f, "
               "\"valu_lanecomp_per_kcyc_simd\": %.4f, \"salu_comp_per_kcyc_simd\": %.4f, "
               "\"valu_gcomp_s\": %.3f}",
               ci ? ", " : "", c.name, blocks, ms, nv ? vc / nv : 0.0, ns ? sc / ns : 0.0, ns ? sdone / ns : 0.0,
               vrate, srate, vdone * 64.0 / (ms * 1e6));
    }
    printf("]}\n");
    return 0;
}
