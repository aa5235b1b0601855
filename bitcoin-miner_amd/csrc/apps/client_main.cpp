// client_main.cpp -- minehip-client: the bitcoin client over LSP.
//
// Reference: bitcoin/client/client.go -- `client <hostport> <message>
// <maxNonce>` (:12-19), connects (:25-29), sends Request(message, 0,
// maxNonce) and prints the server's Result as "Result <hash> <nonce>"
// (printResult, :41-43), or "Disconnected" (:46-48) when the server is lost
// first (:33-37 are TODO in the reference).
#include <stdio.h>
#include <string.h>

#include <vector>

#include "../../../include/minehip.h"
#include "common.hpp"

int main(int argc, char** argv) {
    if (argc != 4) {
        printf("Usage: ./%s <hostport> <message> <maxNonce>", argv[0]);  // client.go:12-15
        return 2;
    }
    uint64_t max_nonce = 0;
    if (!apps::parse_u64(argv[3], &max_nonce)) {
        printf("%s is not a number.\n", argv[3]);  // client.go:18-20
        return 2;
    }
    const lsp_params p = apps::params_from_env();
    lsp_client* c = nullptr;
    int rc = lsp_client_new(argv[1], &p, &c);
    if (rc != LSP_OK) {
        printf("Failed to connect to server: %s\n", apps::lsp_strerror(rc));  // client.go:26-28
        return 1;
    }
    std::vector<char> req(256 + 6 * strlen(argv[2]));
    size_t rn = 0;
    mh_msg_encode(1, (const uint8_t*)argv[2], strlen(argv[2]), 0, max_nonce, 0, 0, req.data(), req.size(), &rn);
    if (lsp_client_write(c, (const uint8_t*)req.data(), rn) != LSP_OK) {
        printf("Disconnected\n");
        lsp_client_close(c);
        return 0;
    }
    std::vector<uint8_t> buf(1 << 16);
    for (;;) {
        size_t n = 0;
        rc = lsp_client_read(c, buf.data(), buf.size(), &n, -1);
        if (rc == LSP_ESHORT) {
            buf.resize(n);
            continue;
        }
        if (rc != LSP_OK) {
            printf("Disconnected\n");  // printDisconnected
            break;
        }
        mh_message m;
        uint8_t data[1];
        const int dr = mh_msg_decode((const char*)buf.data(), n, &m, data, 0);
        if ((dr == MH_OK || dr == MH_ETOOLONG) && m.type == 2) {
            printf("Result %llu %llu\n", (unsigned long long)m.hash, (unsigned long long)m.nonce);  // printResult
            break;
        }
    }
    fflush(stdout);
    lsp_client_close(c);
    return 0;
}
