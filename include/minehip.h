/*
 * minehip.h -- C-ABI of libminehip.so, the MI355X (gfx950) SHA-256 nonce-search
 * backend for the CMU 15-440 bitcoin miner (jack-nie/bitcoin-miner).
 *
 * The reference hot path this library replaces (line numbers into the
 * reference repository):
 *   - bitcoin/hash.go:13-17   func Hash(msg string, nonce uint64) uint64
 *       = BigEndian.Uint64(sha256(fmt.Sprintf("%s %d", msg, nonce))[:8])
 *   - bitcoin/miner/miner.go:33  the miner's scan loop (a TODO stub in the
 *       reference; specification in SURVEY.md §8(a) row A2): over the
 *       inclusive range [Lower, Upper] of a Request (bitcoin/message.go:18-34)
 *       return the first strict-< minimum, i.e. the lexicographic minimum of
 *       (hash, nonce), which becomes a Result (bitcoin/message.go:38-44).
 *
 * A Go miner binds these through cgo; the Python
 * package bitcoin-miner_amd/minehip binds them through ctypes.
 *
 * Conventions for every entry point:
 *   - Plain pointers and sizes; no torch / HIP types cross the ABI.
 *   - The caller owns every buffer.  `msg` is read (and copied) during the
 *     call only; the library never keeps a caller pointer nor hands out
 *     memory the caller must free.
 *   - Return 0 on success or a negative MH_E* code; mh_last_error() then
 *     describes the failure of the calling thread's last call.
 *   - Blocking.  Each call selects its device itself, so one OS thread per
 *     device may call concurrently (the cgo wrapper pins one goroutine per
 *     device with runtime.LockOSThread).
 *   - No CPU fallback: when no usable gfx950 device is present the search
 *     functions fail with MH_ENODEV instead of computing on the host.
 */
#ifndef MINEHIP_H
#define MINEHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error codes (negative returns). */
#define MH_OK 0
#define MH_EINVAL (-1)   /* NULL output pointer, bad device index, ...      */
#define MH_ERANGE (-2)   /* lower > upper                                   */
#define MH_ETOOLONG (-3) /* len(msg) > MH_MAX_MSG_LEN                       */
#define MH_ENODEV (-4)   /* no HIP device / not gfx950                      */
#define MH_EHIP (-5)     /* a HIP runtime call failed (see mh_last_error)   */
#define MH_ENOTREQ (-6)  /* mh_miner_handle: the payload is not a JSON Request */
#define MH_EINTERNAL (-7) /* a launch-plan invariant failed (a library bug)  */
#define MH_EREJECTED (-8) /* mh_server_read: a client's Request was refused  */

/* Longest accepted message.  The LSP transport caps a datagram at 1000 bytes
 * (lsp/util.go:16, lsp/client_impl.go:203), i.e. ~600 bytes of Data after
 * JSON framing; the kernels themselves accept any length (the full 64-byte
 * blocks of "msg " are absorbed into a host midstate). */
#define MH_MAX_MSG_LEN (1u << 20)

/* ABI version of this header, returned by mh_abi_version(). */
#define MH_ABI_VERSION 5

int mh_abi_version(void);

/* Number of HIP devices this process can see (0 when none).  Replaces nothing
 * in the reference; lets the caller size its per-device goroutines. */
int mh_device_count(void);

/* Lexicographic min of (Hash(msg, n), n) over n in [lower, upper] (inclusive,
 * upper may be 2^64-1) on device `dev`.
 * Replaces the miner scan loop over bitcoin.Hash (miner.go:33 spec over
 * hash.go:13-17); *out_hash / *out_nonce are Result.Hash / Result.Nonce
 * (message.go:38-44). */
int mh_search(int dev, const uint8_t *msg, size_t len, uint64_t lower, uint64_t upper,
              uint64_t *out_hash, uint64_t *out_nonce);

/* Same result, the range split over the listed devices, one host thread + HIP
 * stream per listed device, merged on the host by the same lexicographic min
 * (associative, so bit-exact with mh_search).  No device-to-device traffic:
 * each span returns one 16-byte (hash, nonce).
 *   chunk == 0 (adaptive): one contiguous shard per device, sized in
 *     proportion to the device's measured rate (kept per process across
 *     calls; equal shards until measured), so each device runs one search.
 *     A range of >= 2^35 nonces per device keeps its last 1/16 back as 2
 *     chunks per device, handed out as the shards finish (mh_multi_plan
 *     shows the split).
 *   chunk > 0: fixed chunks of that many nonces from the server's scheduler
 *     (include/minehip_server.h).
 * A device that fails hands its shard or chunk back to the others; the call
 * fails only if every device fails (with the first failure's code).  A list
 * may repeat a device (its searches then run one after the other). */
int mh_search_multi(const int *devs, int ndev, const uint8_t *msg, size_t len, uint64_t lower,
                    uint64_t upper, uint64_t chunk, uint64_t *out_hash, uint64_t *out_nonce);

/* Most entries a device list of mh_search_multi / mh_multi_plan may have (one host thread each;
 * a device may be listed more than once). */
#define MH_MAX_WORKERS 256

/* out_hashes[i] = Hash(msg, nonces[i]) computed on device `dev` -- the batched
 * GPU form of bitcoin.Hash (hash.go:13-17).  n may be 0. */
int mh_hash_batch(int dev, const uint8_t *msg, size_t len, const uint64_t *nonces, size_t n,
                  uint64_t *out_hashes);

/* Thread-local description of the calling thread's last failure ("" if none). */
const char *mh_last_error(void);

/* ---- miner process (bitcoin/miner/miner.go, bitcoin/message.go) -------- */

/* bitcoin.Message (message.go:18-23).  type: 0 Join, 1 Request, 2 Result
 * (message.go:7-13). */
typedef struct mh_message {
    int64_t type;
    uint64_t lower, upper;
    uint64_t hash, nonce;
    size_t data_len; /* bytes of Data (UTF-8) */
} mh_message;

/* Go json.Marshal of bitcoin.Message{type, data, lower, upper, hash, nonce},
 * byte for byte: {"Type":..,"Data":"..","Lower":..,"Upper":..,"Hash":..,
 * "Nonce":..} with Go's string escaping (HTML-safe, invalid UTF-8 ->
 * \ufffd).  *out_len receives the needed size; MH_EINVAL if cap is short. */
int mh_msg_encode(int64_t type, const uint8_t *data, size_t dlen, uint64_t lower, uint64_t upper,
                  uint64_t hash, uint64_t nonce, char *out, size_t cap, size_t *out_len);

/* Go json.Unmarshal into bitcoin.Message: case-insensitive keys, unknown
 * keys ignored.  Data (UTF-8) is copied to data[0..data_len); MH_ETOOLONG
 * if data_cap is short (out->data_len still set), MH_EINVAL on bad JSON. */
int mh_msg_decode(const char *json, size_t len, mh_message *out, uint8_t *data, size_t data_cap);

/* One step of the GPU miner (miner.go:33 TODO, spec SURVEY.md §8(a) A2):
 * decode a Request payload, search [Lower, Upper] on the listed devices,
 * encode NewResult(hash, nonce) (message.go:38-44) into out.  The Go miner
 * wraps this between lsp.Client.Read and lsp.Client.Write.  MH_ENOTREQ when
 * the payload is not a JSON bitcoin.Message of type Request, MH_ERANGE when
 * its Lower > Upper: a miner skips those.  Any other error comes from the
 * search itself (MH_EHIP, MH_EINTERNAL, ...): the miner should exit, so the
 * server's lost-miner path hands the chunk to another miner. */
int mh_miner_handle(const int *devs, int ndev, const char *request, size_t len, char *out, size_t cap,
                    size_t *out_len);

/* ---- measurement (no reference counterpart; used by bench.py) ---------- */

/* Enable (on != 0: counters reset) or disable (counters kept, readable) the
 * HIP-event timing of every search-kernel launch on `dev`'s stream. */
int mh_profile_enable(int dev, int on);

/* Counters since the last mh_profile_enable(dev, 1):
 *   out[0] launches of the dominant (fast search) kernel
 *   out[1] nonces those launches processed
 *   out[2] summed kernel duration, nanoseconds (HIP events on the lib's stream)
 *   out[3] algorithmic VALU instructions of those launches: per piece,
 *          nonces x mh_piece.nonce_ops (the nonce-dependent SHA-256 work,
 *          DESIGN.md §4); x64 lanes = int32 lane-ops
 *   out[4] nonces processed by the generic (edge) kernel
 *   out[5] generic kernel duration, nanoseconds
 *   out[6] the same fast-kernel work in SIMD-32 issue slots: per piece,
 *          nonces x mh_piece.nonce_slots (the roofline unit)
 * n = number of slots the caller provides (<= 8). */
int mh_profile_read(int dev, uint64_t *out, int n);

/* Per fast_search<J, MODE> variant and lane length L (lo_digits: 10^L
 * nonces per lane) counters since mh_profile_enable(dev, 1); the roofline's
 * "dominant kernel" is the entry with the largest ns.  The kernel name in a
 * rocprofv3 trace is `mh::fast_search<word, mode>` for every L (the trace
 * tells the launches apart by grid size).  ABI 3 appended lo_digits. */
typedef struct mh_kernel_stat {
    int32_t word, mode;
    uint64_t launches, nonces, ns, ops, slots;
    int32_t lo_digits, reserved;
} mh_kernel_stat;

/* Writes up to cap variants that ran; returns how many ran (or MH_E*). */
int mh_profile_kernels(int dev, mh_kernel_stat *out, int cap);

/* gfx950 VALU instructions of one full SHA-256 compression with no work
 * hoisted (64 rounds x 14 + 48 schedule words x 10). */
#define MH_OPS_PER_BLOCK 1376u

/* ---- introspection (host only, no GPU needed; used by CPU tests) -------- */

/* One piece of a search plan: [first, first+count-1] covered by one kernel. */
typedef struct mh_piece {
    uint64_t first;
    uint64_t count;
    int32_t kind;       /* 0 = fast run kernel, 1 = generic per-nonce kernel */
    int32_t digits;     /* decimal digits of every nonce in the piece */
    int32_t lo_digits;  /* fast: digits enumerated inside a run (L)        */
    int32_t word;       /* fast: message word of the per-nonce digit (J): the last digit's, or
                           (modes 3..5) the word before it, whose last byte is then the digit
                           enumerated innermost (ABI 5) */
    int32_t mode;       /* fast: 0 one block, 1 prefix block per run, 2 two blocks per nonce;
                           3, 4, 5 the same with the innermost digit in word J (ABI 5) */
    int32_t blocks;     /* tail blocks hashed per nonce in the final message */
    uint32_t nonce_ops; /* fast: algorithmic VALU instructions per nonce */
    uint32_t nonce_slots; /* fast: the same work in SIMD-32 issue slots */
} mh_piece;

/* Plan the search of [lower, upper] for `msg`: writes the pieces in
 * increasing nonce order to out (may be NULL) and returns how many there are,
 * or cap + 1 when the plan has more than cap pieces (the first cap written),
 * or a negative MH_E* code. */
int64_t mh_plan(const uint8_t *msg, size_t len, uint64_t lower, uint64_t upper, mh_piece *out, int64_t cap);

/* One span of mh_search_multi's adaptive split (chunk == 0), ABI 4. */
typedef struct mh_span {
    uint64_t lower, upper; /* inclusive */
    int32_t worker;        /* head shard: index into devs; tail chunk: -1 */
    int32_t kind;          /* 0 head shard, 1 tail chunk (handed to the first free worker) */
    double cost;           /* relative cost (issue slots): shards ~ weights */
} mh_span;

/* Host only: how mh_search_multi(chunk = 0) would split [lower, upper] over
 * ndev workers whose rates are in proportion to weights[0..ndev) (> 0; NULL =
 * equal).  Head shards (worker order, empty ones omitted), then tail chunks
 * (nonce order); together they tile [lower, upper] exactly once.  Returns the
 * span count (cap + 1 style truncation as mh_plan) or MH_E*. */
int64_t mh_multi_plan(const uint8_t *msg, size_t len, uint64_t lower, uint64_t upper, const double *weights,
                      int ndev, mh_span *out, int64_t cap);

/* The per-process rate table mh_search_multi sizes its shards by: out[i] =
 * devs[i]'s measured rate in cost units per ns (0 = not measured yet). */
int mh_multi_rates(const int *devs, int ndev, double *out);

#ifdef __cplusplus
}
#endif

#endif /* MINEHIP_H */
