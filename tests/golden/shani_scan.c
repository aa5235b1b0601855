/* shani_scan.c -- fixture generator for the configs[3] full-range answer
 * (tests/golden/fullsize_cfg4.json).  TEST INFRASTRUCTURE: never linked into
 * libminehip.so or loaded by the product path, and never run on the GPU box.
 *
 * BASELINE.json configs[3] scans "cmu440" over [0, 2^40-1]: ~1.1e12 nonces,
 * about 4 h for fullsize_scan.c (OpenSSL, one context copy + Update + Final
 * per nonce) on this container's 8 cores.  This scanner runs the SHA-256
 * compression on the x86 SHA extensions directly (sha256rnds2 / sha256msg1 /
 * sha256msg2), two independent nonces interleaved per thread (measured fastest of 1-8 here), so the scan
 * fits in about an hour.  It is a third SHA-256 implementation: neither the
 * GPU kernels nor oracle/sha256_oracle.c nor OpenSSL.  gen_cfg4.py checks it
 * against OpenSSL (fullsize_cfg2.json chunks, the fullsize_cfg4s.json samples)
 * before its answers are used.
 *
 * Semantics restated (reference, read-only at /root/reference):
 *   Hash(msg, nonce) = BigEndian.Uint64(sha256(fmt.Sprintf("%s %d", msg, nonce))[:8])
 *       bitcoin/hash.go:13-17
 *   scan = first strict-< minimum in increasing nonce order over [lo, hi]
 *       SURVEY.md §8(a) A2 (reference stub bitcoin/miner/miner.go:33)
 * Restricted to messages whose "msg " ‖ digits ‖ padding fits one 64-byte
 * block (len(msg) + 1 + 20 + 9 <= 64), which covers "cmu440" at every nonce.
 *
 * Usage: shani_scan <msg-hex> <lo> <hi> <chunk_bits> <threads> [done-file]
 *   Prints one line "lo hi hash nonce" per 2^chunk_bits chunk as it finishes
 *   (unordered), flushed, so an interrupted run can be resumed: chunks whose
 *   "lo" already appears in done-file are skipped.
 */
#define _GNU_SOURCE
#include <immintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define LANES 2

static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
static const uint32_t IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                               0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

static unsigned char g_prefix[64]; /* "msg " */
static int g_plen;
static uint64_t g_lo, g_hi, g_nchunks;
static int g_bits;
static uint64_t g_next;
static unsigned char* g_skip; /* chunk already in the done-file */
static pthread_mutex_t g_out_mu = PTHREAD_MUTEX_INITIALIZER;

/* H0 << 32 | H1 of one padded block per lane (blk[l]: 64 message bytes). */
__attribute__((target("sha,sse4.1,ssse3"))) static void hash4(const unsigned char* const blk[LANES],
                                                              uint64_t out[LANES]) {
    const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
    /* ABEF / CDGH of the IV: lanes (high..low) A,B,E,F and C,D,G,H */
    const __m128i abef0 = _mm_set_epi32((int)IV[0], (int)IV[1], (int)IV[4], (int)IV[5]);
    const __m128i cdgh0 = _mm_set_epi32((int)IV[2], (int)IV[3], (int)IV[6], (int)IV[7]);
    __m128i s0[LANES], s1[LANES], Q[LANES][4];
#pragma GCC unroll 4
    for (int l = 0; l < LANES; ++l) {
        s0[l] = abef0;
        s1[l] = cdgh0;
#pragma GCC unroll 4
        for (int q = 0; q < 4; ++q) Q[l][q] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(blk[l] + 16 * q)), bswap);
    }
#pragma GCC unroll 16
    for (int q = 0; q < 16; ++q) {
        const __m128i kq = _mm_loadu_si128((const __m128i*)&K256[4 * q]);
#pragma GCC unroll 4
        for (int l = 0; l < LANES; ++l) {
            if (q >= 4) { /* words 4q..4q+3 from quads q-4..q-1 */
                __m128i t = _mm_sha256msg1_epu32(Q[l][q & 3], Q[l][(q - 3) & 3]);
                t = _mm_add_epi32(t, _mm_alignr_epi8(Q[l][(q - 1) & 3], Q[l][(q - 2) & 3], 4));
                Q[l][q & 3] = _mm_sha256msg2_epu32(t, Q[l][(q - 1) & 3]);
            }
            __m128i m = _mm_add_epi32(Q[l][q & 3], kq);
            s1[l] = _mm_sha256rnds2_epu32(s1[l], s0[l], m);
            m = _mm_shuffle_epi32(m, 0x0E);
            s0[l] = _mm_sha256rnds2_epu32(s0[l], s1[l], m);
        }
    }
#pragma GCC unroll 4
    for (int l = 0; l < LANES; ++l) {
        const __m128i f = _mm_add_epi32(s0[l], abef0);
        out[l] = ((uint64_t)(uint32_t)_mm_extract_epi32(f, 3) << 32) | (uint32_t)_mm_extract_epi32(f, 2);
    }
}

static int fmt_dec(uint64_t n, char* out) {
    char tmp[24];
    int k = 0;
    do {
        tmp[k++] = (char)('0' + n % 10);
        n /= 10;
    } while (n);
    for (int i = 0; i < k; ++i) out[i] = tmp[k - 1 - i];
    return k;
}

/* the padded single block of prefix ‖ digits */
static void make_block(const char* dig, int d, unsigned char b[64]) {
    memset(b, 0, 64);
    memcpy(b, g_prefix, (size_t)g_plen);
    memcpy(b + g_plen, dig, (size_t)d);
    const int n = g_plen + d;
    b[n] = 0x80;
    const uint64_t bits = (uint64_t)n * 8;
    for (int i = 0; i < 8; ++i) b[63 - i] = (unsigned char)(bits >> (8 * i));
}

static void scan(uint64_t lo, uint64_t hi, uint64_t* bh, uint64_t* bn) {
    uint64_t best_h = UINT64_MAX, best_n = UINT64_MAX;
    int first = 1;
    char dig[24];
    int d = fmt_dec(lo, dig);
    unsigned char cur[64];   /* block of nonce n, digits edited in place */
    unsigned char lane[LANES][64];
    const unsigned char* blk[LANES];
    make_block(dig, d, cur);
    uint64_t n = lo;
    for (;;) {
        uint64_t nn[LANES], h[LANES];
        int k = 0;
        for (; k < LANES; ++k) {
            memcpy(lane[k], cur, 64);
            blk[k] = lane[k];
            nn[k] = n;
            if (n == hi) {
                ++k;
                break;
            }
            ++n;
            /* ++ of the digits inside the block; a new length rebuilds it */
            int i = g_plen + d - 1;
            while (i >= g_plen && cur[i] == '9') cur[i--] = '0';
            if (i >= g_plen) {
                cur[i]++;
            } else {
                d = fmt_dec(n, dig);
                make_block(dig, d, cur);
            }
        }
        for (int j = k; j < LANES; ++j) blk[j] = lane[0]; /* ragged end: repeat lane 0 */
        hash4(blk, h);
        for (int j = 0; j < k; ++j) /* increasing nonce order, strict < */
            if (first || h[j] < best_h) {
                best_h = h[j];
                best_n = nn[j];
                first = 0;
            }
        if (nn[k - 1] == hi) break;
    }
    *bh = best_h;
    *bn = best_n;
}

static void* worker(void* arg) {
    (void)arg;
    for (;;) {
        const uint64_t i = __atomic_fetch_add(&g_next, 1, __ATOMIC_RELAXED);
        if (i >= g_nchunks) return NULL;
        if (g_skip && g_skip[i]) continue;
        const uint64_t lo = g_lo + (i << g_bits);
        uint64_t hi = lo + ((1ull << g_bits) - 1);
        if (hi > g_hi || hi < lo) hi = g_hi;
        uint64_t h, n;
        scan(lo, hi, &h, &n);
        pthread_mutex_lock(&g_out_mu);
        printf("%llu %llu %llu %llu\n", (unsigned long long)lo, (unsigned long long)hi, (unsigned long long)h,
               (unsigned long long)n);
        fflush(stdout);
        pthread_mutex_unlock(&g_out_mu);
    }
}

static int hexval(int c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    return -1;
}

int main(int argc, char** argv) {
    if (argc != 6 && argc != 7) {
        fprintf(stderr, "usage: %s <msg-hex> <lo> <hi> <chunk_bits> <threads> [done-file]\n", argv[0]);
        return 2;
    }
    const char* hx = argv[1];
    const size_t hl = strlen(hx);
    if (hl % 2 || hl / 2 + 1 + 20 + 9 > 64) {
        fprintf(stderr, "message must fit one block with 20 digits\n");
        return 2;
    }
    for (size_t i = 0; i < hl / 2; ++i) {
        const int a = hexval(hx[2 * i]), b = hexval(hx[2 * i + 1]);
        if (a < 0 || b < 0) return 2;
        g_prefix[i] = (unsigned char)(a * 16 + b);
    }
    g_prefix[hl / 2] = ' ';
    g_plen = (int)(hl / 2 + 1);
    g_lo = strtoull(argv[2], NULL, 10);
    g_hi = strtoull(argv[3], NULL, 10);
    g_bits = atoi(argv[4]);
    const int threads = atoi(argv[5]);
    if (g_lo > g_hi || g_bits < 1 || g_bits > 40 || threads < 1) return 2;
    g_nchunks = ((g_hi - g_lo) >> g_bits) + 1;
    if (argc == 7) {
        g_skip = calloc(g_nchunks, 1);
        FILE* f = fopen(argv[6], "r");
        if (f) {
            unsigned long long a, b, c, e;
            while (fscanf(f, "%llu %llu %llu %llu", &a, &b, &c, &e) == 4)
                if (a >= g_lo && a <= g_hi && ((a - g_lo) & ((1ull << g_bits) - 1)) == 0)
                    g_skip[(a - g_lo) >> g_bits] = 1;
            fclose(f);
        }
    }
    pthread_t* th = malloc(sizeof(pthread_t) * (size_t)threads);
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, worker, NULL);
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    return 0;
}
