/*
 * oracle/openssl_scan.c -- an OPTIMISED CPU scan, for the bench's CPU
 * baseline only.
 *
 * TEST INFRASTRUCTURE ONLY: nothing in the product links, loads or calls this
 * file.  bench.py's cpu_baseline leg times it next to the plain restatement
 * (sha256_oracle.c, kind "port") to show what a tuned CPU miner reaches on the
 * same host.  Same semantics (bitcoin/hash.go:13-17; scan spec SURVEY.md
 * §8(a) A2, reference stub bitcoin/miner/miner.go:33), but, unlike the
 * reference, it absorbs the constant "msg " prefix once into a SHA256_CTX
 * (midstate), keeps the decimal nonce as an ASCII counter, and hashes with
 * OpenSSL's libcrypto (SHA-NI on x86).  Threads take contiguous sub-ranges;
 * the per-thread first minima merge lexicographically.
 */
#define _GNU_SOURCE
#include <openssl/sha.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    const SHA256_CTX *base;
    uint64_t lo, hi, hash, nonce;
} ossl_job;

static int fmt_dec(uint64_t n, char *out) {
    char tmp[24];
    int k = 0;
    do {
        tmp[k++] = (char)('0' + n % 10);
        n /= 10;
    } while (n);
    for (int i = 0; i < k; ++i) out[i] = tmp[k - 1 - i];
    return k;
}

static void *ossl_worker(void *arg) {
    ossl_job *j = (ossl_job *)arg;
    char dig[24];
    int d = fmt_dec(j->lo, dig);
    unsigned char md[32];
    uint64_t bh = UINT64_MAX, bn = j->lo;
    int first = 1;
    for (uint64_t n = j->lo;; ++n) {
        SHA256_CTX c = *j->base;
        SHA256_Update(&c, dig, (size_t)d);
        SHA256_Final(md, &c);
        uint64_t h = 0;
        for (int i = 0; i < 8; ++i) h = (h << 8) | md[i];
        if (first || h < bh) {
            bh = h;
            bn = n;
            first = 0;
        }
        if (n == j->hi) break;
        int i = d - 1; /* ASCII ++ */
        while (i >= 0 && dig[i] == '9') dig[i--] = '0';
        if (i >= 0) {
            dig[i]++;
        } else {
            dig[0] = '1';
            memset(dig + 1, '0', (size_t)d);
            d++;
        }
    }
    j->hash = bh;
    j->nonce = bn;
    return NULL;
}

int oracle_search_openssl(const uint8_t *msg, size_t len, uint64_t lower, uint64_t upper, int nthreads,
                          uint64_t *out_hash, uint64_t *out_nonce) {
    if (lower > upper) return -1;
    if (nthreads < 1) nthreads = 1;
    uint64_t span = upper - lower;
    if (span < (uint64_t)nthreads) nthreads = (int)(span + 1);
    SHA256_CTX base;
    SHA256_Init(&base);
    SHA256_Update(&base, msg, len);
    SHA256_Update(&base, " ", 1);
    ossl_job *jobs = (ossl_job *)calloc((size_t)nthreads, sizeof *jobs);
    pthread_t *tid = (pthread_t *)calloc((size_t)nthreads, sizeof *tid);
    if (!jobs || !tid) {
        free(jobs);
        free(tid);
        return -2;
    }
    uint64_t per = span / (uint64_t)nthreads + 1, cur = lower;
    int used = 0;
    for (int i = 0; i < nthreads; ++i) {
        jobs[i].base = &base;
        jobs[i].lo = cur;
        jobs[i].hi = (upper - cur < per - 1) ? upper : cur + per - 1;
        pthread_create(&tid[i], NULL, ossl_worker, &jobs[i]);
        used++;
        if (jobs[i].hi == upper) break;
        cur = jobs[i].hi + 1;
    }
    uint64_t bh = UINT64_MAX, bn = UINT64_MAX;
    for (int i = 0; i < used; ++i) {
        pthread_join(tid[i], NULL);
        if (i == 0 || jobs[i].hash < bh || (jobs[i].hash == bh && jobs[i].nonce < bn)) {
            bh = jobs[i].hash;
            bn = jobs[i].nonce;
        }
    }
    free(jobs);
    free(tid);
    *out_hash = bh;
    *out_nonce = bn;
    return 0;
}
