// cli.cpp -- native command-line front ends of libminehip (C++ callers of the
// C-ABI in include/minehip.h; no Python, no torch).
//
//   minehip-search <message> <maxNonce> [lower]
//       scans [lower (default 0), maxNonce] on every visible GPU and prints
//       "Result <hash> <nonce>" -- the output format of the reference client
//       (bitcoin/client/client.go:41-43), whose argument convention
//       (client.go:12-19: <message> <maxNonce>) it follows minus the hostport.
//
// The miner, server and client processes over LSP are apps/*_main.cpp.
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/minehip.h"

namespace {

bool parse_u64(const char* s, uint64_t* out) {  // strconv.ParseUint(s, 10, 64)
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

std::vector<int> all_devices() {
    std::vector<int> d;
    for (int i = 0; i < mh_device_count(); ++i) d.push_back(i);
    return d;
}

int run_search(int argc, char** argv) {
    if (argc != 3 && argc != 4) {
        printf("Usage: ./%s <message> <maxNonce> [lower]", argv[0]);
        return 2;
    }
    uint64_t hi = 0, lo = 0;
    if (!parse_u64(argv[2], &hi)) {
        printf("%s is not a number.\n", argv[2]);
        return 2;
    }
    if (argc == 4 && !parse_u64(argv[3], &lo)) {
        printf("%s is not a number.\n", argv[3]);
        return 2;
    }
    const std::vector<int> devs = all_devices();
    if (devs.empty()) {
        fprintf(stderr, "minehip: no HIP device\n");
        return 1;
    }
    uint64_t h = 0, n = 0;
    const int rc = mh_search_multi(devs.data(), (int)devs.size(), (const uint8_t*)argv[1], strlen(argv[1]), lo,
                                   hi, 0, &h, &n);
    if (rc != MH_OK) {
        fprintf(stderr, "minehip: %s\n", mh_last_error());
        return 1;
    }
    printf("Result %llu %llu\n", (unsigned long long)h, (unsigned long long)n);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    return run_search(argc, argv);
}
