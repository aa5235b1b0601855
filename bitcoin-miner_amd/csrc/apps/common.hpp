// common.hpp -- shared bits of the native miner / server / client processes.
#pragma once
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <time.h>

#include "../../../include/lsp440.h"

namespace apps {

// strconv.ParseUint(s, 10, 64) (client.go:16): digits only, no overflow.
inline bool parse_u64(const char* s, uint64_t* out) {
    if (!s || !*s) return false;
    for (const char* p = s; *p; ++p)
        if (*p < '0' || *p > '9') return false;
    errno = 0;
    char* end = nullptr;
    const unsigned long long v = strtoull(s, &end, 10);
    if (errno == ERANGE || *end) return false;
    *out = v;
    return true;
}

// lsp.NewParams() (params.go:34-40), overridable from the environment
// (LSP_EPOCH_LIMIT, LSP_EPOCH_MILLIS, LSP_WINDOW_SIZE) so tests can detect a
// lost peer in a second instead of EpochLimit x 2 s.
inline lsp_params params_from_env() {
    lsp_params p;
    lsp_default_params(&p);
    if (const char* e = getenv("LSP_EPOCH_LIMIT")) p.epoch_limit = atoi(e);
    if (const char* e = getenv("LSP_EPOCH_MILLIS")) p.epoch_millis = atoi(e);
    if (const char* e = getenv("LSP_WINDOW_SIZE")) p.window_size = atoi(e);
    return p;
}

inline const char* lsp_strerror(int rc) {
    switch (rc) {
        case LSP_ECLOSED: return "connection closed";
        case LSP_ELOST: return "connection lost";
        case LSP_ECONNECT: return "can not establish connection";  // lsp/util.go:12
        case LSP_ETIMEOUT: return "timeout";
        case LSP_EINVAL: return "invalid argument";
        case LSP_ESOCK: return "socket error";
        case LSP_ESHORT: return "buffer too small";
        default: return "ok";
    }
}

inline uint64_t now_ns() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

}  // namespace apps
