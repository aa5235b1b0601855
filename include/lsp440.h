/*
 * lsp440.h -- the Live Sequence Protocol (CMU 15-440 P1) in C++, wire
 * compatible with the reference's Go package, exported by liblsp440.so.
 *
 * Why it exists: the miner, server and client processes of the reference
 * talk LSP over UDP (lsp/client_api.go:6-30, lsp/server_api.go:6-39).  The Go
 * toolchain is absent from this image and from the MI355X box, so the native
 * processes that call libminehip (minehip-miner, minehip-server,
 * minehip-client) need their own LSP endpoint.
 * This one speaks the same datagrams as the reference, so a native GPU miner
 * can join a Go server built from the reference and a Go miner can join the
 * native server:
 *   - one datagram = Go encoding/json of lsp.Message{Type, ConnID, SeqNum,
 *     Size, Payload} (lsp/message.go:17-24, lsp/util.go:19-33), Payload as
 *     base64, nil as null; Type 0 Connect, 1 Data, 2 Ack (message.go:10-14);
 *   - Params{EpochLimit 5, EpochMillis 2000, WindowSize 1} defaults
 *     (lsp/params.go:8-12);
 *   - Connect -> Ack(connID, 0); Data seq numbers from 1 per direction,
 *     each acked, delivered in order exactly once; at most WindowSize
 *     unacked Data messages in flight; a Data whose payload is shorter than
 *     its Size is dropped, a longer one truncated to Size;
 *   - every epoch: resend Connect (until acked), resend unacked Data, send
 *     Ack(connID, 0) while no Data has arrived, else re-ack the last
 *     WindowSize Data messages; a peer silent for more than EpochLimit epochs
 *     is lost (lsp/client_impl.go:216-226, server_impl.go:165-173).
 *
 * the reference server marks a lost client internally
 * but never surfaces it (server_impl.go:165-173 returns without telling
 * Read), so its Read cannot report `(connID, err)` as server_api.go:7-17
 * requires and dropped-miner recovery never starts.  Here Read returns
 * (connID, LSP_ELOST) once that client's already-received messages are read.
 *
 * A server connection whose loss or close Read has reported is freed; later
 * write / close_conn on its id return LSP_ELOST / LSP_ECLOSED.
 *
 * Every call is thread-safe; each endpoint runs one background thread.
 * Return codes: 0 ok, negative LSP_E*.  Buffers are caller-owned.
 */
#ifndef LSP440_H
#define LSP440_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LSP_OK 0
#define LSP_ECLOSED -10  /* closed explicitly (ErrConnClosed, lsp/util.go:10)           */
#define LSP_ELOST -11    /* epoch limit reached: the peer is lost                         */
#define LSP_ECONNECT -12 /* no Ack to Connect within EpochLimit epochs (util.go:12)       */
#define LSP_ETIMEOUT -13 /* a read with a timeout expired (test convenience)              */
#define LSP_EINVAL -14   /* bad argument / unknown connID                                 */
#define LSP_ESOCK -15    /* socket / address error                                        */
#define LSP_ESHORT -16   /* caller's buffer too small; *len = the payload size, kept      */
#define LSP_ETOOBIG -17  /* write: the Data datagram would exceed LSP_MAX_DATAGRAM        */

/* Largest datagram a write may produce (the UDP/IPv4 payload limit); a larger
 * frame could never be delivered, so write refuses it with LSP_ETOOBIG
 * instead of resending it forever.  Interop note: the reference's Go peers
 * read at most MaxMessageSize = 1000 bytes per datagram (lsp/util.go:16,
 * lsp/client_impl.go:203), i.e. about 600 bytes of payload after JSON and
 * base64 framing; frames between 1000 and LSP_MAX_DATAGRAM bytes only reach
 * liblsp440 peers. */
#define LSP_MAX_DATAGRAM 65507

typedef struct lsp_params {
    int epoch_limit;  /* Params.EpochLimit  */
    int epoch_millis; /* Params.EpochMillis */
    int window_size;  /* Params.WindowSize  */
} lsp_params;

/* lsp.NewParams() (params.go:34-40). */
void lsp_default_params(lsp_params *p);

/* ---- client (lsp/client_api.go) ---------------------------------------- */
typedef struct lsp_client lsp_client;

/* lsp.NewClient(hostport, params): blocks until the server acked Connect, or
 * returns LSP_ECONNECT after EpochLimit epochs.  params NULL = defaults. */
int lsp_client_new(const char *hostport, const lsp_params *params, lsp_client **out);
/* Client.ConnID(). */
int lsp_client_conn_id(lsp_client *c);
/* Client.Read(): the next in-order payload.  Blocks (timeout_ms < 0) or waits
 * at most timeout_ms (LSP_ETIMEOUT).  LSP_ELOST / LSP_ECLOSED once nothing
 * received is left to return. */
int lsp_client_read(lsp_client *c, uint8_t *buf, size_t cap, size_t *len, int timeout_ms);
/* Client.Write(payload): non-blocking; LSP_ELOST / LSP_ECLOSED when the
 * connection is gone. */
int lsp_client_write(lsp_client *c, const uint8_t *payload, size_t len);
/* Client.Close(): blocks until every written message is acked (or the server
 * is lost), stops the endpoint and frees it.  Returns LSP_ELOST if the server
 * was lost with messages unacked. */
int lsp_client_close(lsp_client *c);

/* ---- server (lsp/server_api.go) ---------------------------------------- */
typedef struct lsp_server lsp_server;

/* lsp.NewServer(port, params): binds UDP :port (0 = any free port, see
 * lsp_server_port) and returns at once. */
int lsp_server_new(int port, const lsp_params *params, lsp_server **out);
int lsp_server_port(lsp_server *s);
/* Server.Read(): (connID, payload).  Returns LSP_OK with data, or
 * LSP_ELOST / LSP_ECLOSED with *conn_id = the client that was lost / closed
 * (after its received messages), or LSP_ECLOSED with *conn_id = 0 once the
 * server is closed.  timeout_ms as lsp_client_read. */
int lsp_server_read(lsp_server *s, int *conn_id, uint8_t *buf, size_t cap, size_t *len, int timeout_ms);
/* Server.Write(connID, payload): non-blocking. */
int lsp_server_write(lsp_server *s, int conn_id, const uint8_t *payload, size_t len);
/* Server.CloseConn(connID): non-blocking; pending messages are still sent. */
int lsp_server_close_conn(lsp_server *s, int conn_id);
/* Server.Close(): blocks until every client's pending messages are acked,
 * stops the endpoint and frees it; LSP_ELOST if some client was lost. */
int lsp_server_close(lsp_server *s);

/* ---- fault injection for tests (the reference's lspnet/staff.go) -------- */
/* Percent (0..100) of datagrams dropped on read / write, per side. */
void lsp_set_drop_percent(int client_read, int client_write, int server_read, int server_write);
/* Percent of Data datagrams whose payload is cut to half / padded with extra
 * bytes on write (Size unchanged), as lspnet's shortening/lengthening. */
void lsp_set_msg_mangle_percent(int shorten, int lengthen);

/* ---- wire codec (exported for tests) ----------------------------------- */
/* json.Marshal(lsp.Message): writes at most cap bytes, *len = full size;
 * LSP_ESHORT if cap is too small.  payload NULL with has_payload 0 = null. */
int lsp_marshal(int type, int64_t conn_id, int64_t seq, int64_t size, const uint8_t *payload, size_t plen,
                int has_payload, char *out, size_t cap, size_t *len);
/* json.Unmarshal into lsp.Message: LSP_EINVAL if not such an object. */
int lsp_unmarshal(const char *js, size_t jlen, int *type, int64_t *conn_id, int64_t *seq, int64_t *size,
                  uint8_t *payload, size_t cap, size_t *plen, int *has_payload);

#ifdef __cplusplus
}
#endif
#endif /* LSP440_H */
