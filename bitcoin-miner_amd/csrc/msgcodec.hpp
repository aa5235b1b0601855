// msgcodec.hpp -- Go encoding/json codec of bitcoin.Message (message.go:18-23),
// shared by the miner handler (message.cpp) and the server (server.cpp).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>

namespace mh {

int set_error(int code, const char* what);

// bitcoin.Message; type 0 Join, 1 Request, 2 Result (message.go:7-13).
struct Msg {
    int64_t type = 0;
    std::string data;
    uint64_t lower = 0, upper = 0, hash = 0, nonce = 0;
};

// json.Unmarshal into Message: false when the payload is not a JSON object of it.
bool decode(const char* js, size_t len, Msg* m);

// json.Marshal of Message, byte for byte.
std::string encode(int64_t type, const uint8_t* data, size_t dlen, uint64_t lower, uint64_t upper, uint64_t hash,
                   uint64_t nonce);

}  // namespace mh
