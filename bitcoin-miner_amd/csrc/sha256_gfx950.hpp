// sha256_gfx950.hpp -- SHA-256 (FIPS 180-4) compression written for the
// gfx950 VALU.
//
// Reference semantics: Go crypto/sha256 as called by bitcoin/hash.go:14-16.
//
// Instruction mapping (verified in the .s):
//   rotr        -> v_alignbit_b32 x, x, n           (1 op)
//   a ^ b ^ c   -> v_bitop3_b32 ... bitop3:0x96     (1 op; gfx950 has no v_xor3_b32)
//   Maj(a,b,c)  -> v_bitop3_b32 ... bitop3:0xe8     (1 op)
//   Ch(e,f,g)   -> v_bitop3_b32 ... bitop3:0xca     (1 op)
//   3-way adds  -> v_add3_u32                        (1 op)
// giving 14 VALU ops per round and 10 per message-schedule word.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mh {
namespace dev {

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}
// bitop3 truth-table index is (src0 << 2) | (src1 << 1) | src2; e ? f : g -> 0xCA.
// Written as the builtin so the compiler cannot split it into (e&f) + (~e&g)
// and spread the halves over the add chain (2 ops instead of 1).
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) {
    return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
}
__device__ __forceinline__ uint32_t bsig0(uint32_t a) { return xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)); }
__device__ __forceinline__ uint32_t bsig1(uint32_t e) { return xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)); }
__device__ __forceinline__ uint32_t ssig0(uint32_t x) { return xor3(rotr(x, 7), rotr(x, 18), x >> 3); }
__device__ __forceinline__ uint32_t ssig1(uint32_t x) { return xor3(rotr(x, 17), rotr(x, 19), x >> 10); }

// FIPS 180-4 §4.2.2 constants; every use is at a compile-time index after
// unrolling, so they become scalar operands (K lives in SGPRs, never memory).
#define MH_K256                                                                                     \
    {0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,      \
     0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,      \
     0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,      \
     0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,      \
     0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,      \
     0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,      \
     0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,      \
     0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,      \
     0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,      \
     0xc67178f2u}

// Full compression with feed-forward: st <- st + rounds(st, in).
__device__ __forceinline__ void sha256_block(uint32_t st[8], const uint32_t in[16]) {
    constexpr uint32_t K[64] = MH_K256;
    uint32_t w[64];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = in[i];
#pragma unroll
    for (int i = 16; i < 64; ++i) w[i] = (w[i - 16] + w[i - 7]) + ssig0(w[i - 15]) + ssig1(w[i - 2]);
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        const uint32_t t1 = h + bsig1(e) + ch(e, f, g) + (K[i] + w[i]);
        const uint32_t t2 = bsig0(a) + maj(a, b, c);
        h = g; g = f; f = e; e = d + t1;
        d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// Compression that only produces what Hash() reads: the first two output
// words H0 = st0 + a64 and H1 = st1 + a63 (bitcoin/hash.go:16 keeps digest
// bytes 0..7).  The e-update of the last round and the other six
// feed-forward adds are dead and vanish.
__device__ __forceinline__ void sha256_block_h01(const uint32_t st[8], const uint32_t in[16], uint32_t& h0,
                                                 uint32_t& h1) {
    uint32_t s[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = st[i];
    sha256_block(s, in);
    h0 = s[0];
    h1 = s[1];
}

}  // namespace dev
}  // namespace mh
