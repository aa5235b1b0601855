/* fullsize_scan.c -- fixture generator for the full-size scan answers
 * (tests/golden/fullsize_*.json).  TEST INFRASTRUCTURE: never linked into
 * libminehip.so or loaded by the product path.
 *
 * Computes, for one message and an inclusive nonce range, the lexicographic
 * (hash, nonce) minimum of every 2^chunk_bits slice and of the whole range,
 * with OpenSSL's SHA-256 (libcrypto 3; SHA-NI on x86) -- an implementation
 * independent both of the GPU kernels and of oracle/sha256_oracle.c, so the
 * fixtures pin the product at BASELINE.json's full sizes without routing
 * through our own CPU restatement.
 *
 * Semantics restated (reference, read-only at /root/reference):
 *   Hash(msg, nonce) = BigEndian.Uint64(sha256(fmt.Sprintf("%s %d", msg, nonce))[:8])
 *       bitcoin/hash.go:13-17
 *   scan = first strict-< minimum in increasing nonce order over [lo, hi]
 *       SURVEY.md §8(a) A2 (reference stub bitcoin/miner/miner.go:33)
 * The constant "msg " prefix is absorbed once into a SHA256_CTX that every
 * nonce copies; the digits are kept as an ASCII counter and incremented.
 *
 * Build / run: see tests/golden/gen_fullsize.py (gcc -O2 ... -lcrypto -lpthread).
 * Output: one JSON object on stdout.
 */
#define _GNU_SOURCE
#include <openssl/sha.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    uint64_t hash, nonce;
} best_t;

static const unsigned char* g_msg;
static size_t g_len;
static uint64_t g_lo, g_hi, g_nchunks;
static int g_bits;
static best_t* g_res;
static uint64_t g_next;  /* next chunk index (atomic) */
static SHA256_CTX g_base;

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

/* ++ of an ASCII decimal string of length *len (no leading zeros) */
static void inc_dec(char* s, int* len) {
    int i = *len - 1;
    while (i >= 0 && s[i] == '9') s[i--] = '0';
    if (i >= 0) {
        s[i]++;
    } else { /* 99..9 -> 100..0 */
        s[0] = '1';
        memset(s + 1, '0', (size_t)*len);
        (*len)++;
    }
}

static best_t scan(uint64_t lo, uint64_t hi) {
    best_t b = {UINT64_MAX, UINT64_MAX};
    int first = 1;
    char dig[24];
    int d = fmt_dec(lo, dig);
    unsigned char md[32];
    for (uint64_t n = lo;; ++n) {
        SHA256_CTX c = g_base;
        SHA256_Update(&c, dig, (size_t)d);
        SHA256_Final(md, &c);
        uint64_t h = 0;
        for (int i = 0; i < 8; ++i) h = (h << 8) | md[i];
        if (first || h < b.hash) { /* strict <, increasing n: the first minimum */
            b.hash = h;
            b.nonce = n;
            first = 0;
        }
        if (n == hi) break;
        inc_dec(dig, &d);
    }
    return b;
}

static void* worker(void* arg) {
    (void)arg;
    for (;;) {
        uint64_t i = __atomic_fetch_add(&g_next, 1, __ATOMIC_RELAXED);
        if (i >= g_nchunks) return NULL;
        uint64_t lo = g_lo + (i << g_bits);
        uint64_t hi = lo + ((1ull << g_bits) - 1);
        if (hi > g_hi || hi < lo) hi = g_hi;
        g_res[i] = scan(lo, hi);
    }
}

static int hexval(int c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    return -1;
}

int main(int argc, char** argv) {
    if (argc != 6) {
        fprintf(stderr, "usage: %s <msg-hex> <lo> <hi> <chunk_bits> <threads>\n", argv[0]);
        return 2;
    }
    const char* hx = argv[1];
    size_t hl = strlen(hx);
    if (hl % 2) return 2;
    unsigned char* m = malloc(hl / 2 + 2);
    for (size_t i = 0; i < hl / 2; ++i) {
        int a = hexval(hx[2 * i]), b = hexval(hx[2 * i + 1]);
        if (a < 0 || b < 0) return 2;
        m[i] = (unsigned char)(a * 16 + b);
    }
    m[hl / 2] = ' ';
    g_msg = m;
    g_len = hl / 2 + 1;
    g_lo = strtoull(argv[2], NULL, 10);
    g_hi = strtoull(argv[3], NULL, 10);
    g_bits = atoi(argv[4]);
    int threads = atoi(argv[5]);
    if (g_lo > g_hi || g_bits < 1 || g_bits > 40 || threads < 1) return 2;
    g_nchunks = ((g_hi - g_lo) >> g_bits) + 1;
    g_res = calloc(g_nchunks, sizeof(best_t));
    SHA256_Init(&g_base);
    SHA256_Update(&g_base, g_msg, g_len);

    pthread_t* th = malloc(sizeof(pthread_t) * (size_t)threads);
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, worker, NULL);
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);

    best_t all = g_res[0];
    for (uint64_t i = 1; i < g_nchunks; ++i)
        if (g_res[i].hash < all.hash || (g_res[i].hash == all.hash && g_res[i].nonce < all.nonce)) all = g_res[i];
    printf("{\"lo\": %llu, \"hi\": %llu, \"chunk_bits\": %d, \"result\": [%llu, %llu], \"chunks\": [",
           (unsigned long long)g_lo, (unsigned long long)g_hi, g_bits, (unsigned long long)all.hash,
           (unsigned long long)all.nonce);
    for (uint64_t i = 0; i < g_nchunks; ++i)
        printf("%s[%llu, %llu]", i ? ", " : "", (unsigned long long)g_res[i].hash,
               (unsigned long long)g_res[i].nonce);
    printf("]}\n");
    return 0;
}
