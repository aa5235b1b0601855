// miner_main.cpp -- minehip-miner: the GPU-backed miner process.
//
// Reference: bitcoin/miner/miner.go -- `miner <hostport>` (:18-24) joins the
// server (joinWithServer, :11-15: lsp.NewClient + Join, message.go:47-49),
// then (:33, TODO in the reference; spec SURVEY.md §8(a) A2) loops: Read a
// Request (message.go:27-34), scan [Lower, Upper], Write NewResult(hash,
// nonce) (message.go:38-44).  A Read error (server lost / closed) ends it.
// The scan is libminehip's mh_miner_handle over every visible GPU (one miner
// process per GPU: HIP_VISIBLE_DEVICES).  LSP is liblsp440 (wire compatible
// with the reference's lsp package, include/lsp440.h).
//
//   minehip-miner <hostport>     the miner over LSP
//   minehip-miner --stdio        the per-message step alone: one JSON
//                                Message per stdin line -> Result line
#include <stdio.h>
#include <string.h>

#include <iostream>
#include <string>
#include <vector>

#include "../../../include/minehip.h"
#include "common.hpp"

namespace {

std::vector<int> all_devices() {
    std::vector<int> d;
    for (int i = 0; i < mh_device_count(); ++i) d.push_back(i);
    return d;
}

int run_stdio(const std::vector<int>& devs) {
    std::string line;
    char out[256];
    while (std::getline(std::cin, line)) {
        size_t n = 0;
        const int rc = mh_miner_handle(devs.data(), (int)devs.size(), line.data(), line.size(), out, sizeof out, &n);
        if (rc == MH_ENOTREQ || rc == MH_ERANGE) continue;  // not a (valid) Request: ignored
        if (rc != MH_OK) {
            fprintf(stderr, "minehip: %s\n", mh_last_error());
            return 1;
        }
        fwrite(out, 1, n, stdout);
        fputc('\n', stdout);
        fflush(stdout);
    }
    return 0;
}

int run_lsp(const char* hostport, const std::vector<int>& devs) {
    const lsp_params p = apps::params_from_env();
    lsp_client* c = nullptr;
    int rc = lsp_client_new(hostport, &p, &c);  // joinWithServer (miner.go:11-15)
    if (rc != LSP_OK) {
        printf("Failed to join with server: %s\n", apps::lsp_strerror(rc));
        return 1;
    }
    char join[128];
    size_t jn = 0;
    mh_msg_encode(0, nullptr, 0, 0, 0, 0, 0, join, sizeof join, &jn);  // NewJoin()
    if (lsp_client_write(c, (const uint8_t*)join, jn) != LSP_OK) {
        lsp_client_close(c);
        return 1;
    }
    std::vector<uint8_t> buf(1 << 16);
    char out[256];
    int status = 0;
    for (;;) {
        size_t n = 0;
        rc = lsp_client_read(c, buf.data(), buf.size(), &n, -1);
        if (rc == LSP_ESHORT) {
            buf.resize(n);
            continue;
        }
        if (rc != LSP_OK) break;  // server lost or closed: the miner is done
        size_t on = 0;
        const int hr = mh_miner_handle(devs.data(), (int)devs.size(), (const char*)buf.data(), n, out, sizeof out,
                                       &on);
        if (hr == MH_ENOTREQ || hr == MH_ERANGE) {  // not a Request, or Lower > Upper: no answer
            fprintf(stderr, "minehip-miner: ignored a message: %s\n", mh_last_error());
            continue;
        }
        if (hr != MH_OK) {  // the search failed: leave, so the server reassigns the chunk
            fprintf(stderr, "minehip-miner: %s\n", mh_last_error());
            status = 1;
            break;
        }
        if (lsp_client_write(c, (const uint8_t*)out, on) != LSP_OK) break;
    }
    lsp_client_close(c);
    return status;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc != 2) {
        printf("Usage: ./%s <hostport>", argv[0]);  // miner.go:19-21
        return 2;
    }
    const std::vector<int> devs = all_devices();
    if (devs.empty()) {
        fprintf(stderr, "minehip: no HIP device\n");
        return 1;
    }
    if (!strcmp(argv[1], "--stdio")) return run_stdio(devs);
    return run_lsp(argv[1], devs);
}
