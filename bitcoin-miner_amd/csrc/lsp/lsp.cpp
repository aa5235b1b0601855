// lsp.cpp -- the Live Sequence Protocol endpoint behind include/lsp440.h.
//
// Behaviour follows the reference's LSP contract and its implementation
// (line numbers into /root/reference):
//   lsp/message.go:10-24     message types and fields (the JSON wire form)
//   lsp/util.go:19-33        json.Marshal / json.Unmarshal per datagram
//   lsp/params.go:8-12       EpochLimit 5, EpochMillis 2000, WindowSize 1
//   lsp/client_impl.go:56-125  NewClient: Connect, resent every epoch, until
//                            Ack(connID, 0) or more than EpochLimit epochs
//   lsp/client_impl.go:203-327 acks, in-order delivery, sliding window,
//                            epoch resends (resendAckMessages :360-369)
//   lsp/server_impl.go:59-148  Connect -> new connID + Ack; Data -> Ack
//   lsp/client_api.go, lsp/server_api.go  Read/Write/Close semantics
// One background thread per endpoint runs poll() over the UDP socket and an
// eventfd, and ticks the epoch; API calls take the endpoint mutex and send
// directly.  No Go-style channel graph: a single state machine per endpoint.
#include <arpa/inet.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <poll.h>
#include <string.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/lsp440.h"

namespace lsp440 {
namespace {

enum MsgType { kConnect = 0, kData = 1, kAck = 2 };
constexpr size_t kMaxDatagram = LSP_MAX_DATAGRAM;

struct Wire {
    int type = 0;
    int64_t conn = 0, seq = 0, size = 0;
    bool has_payload = false;
    std::string payload;
};

// ---- Go encoding/json of lsp.Message -----------------------------------
const char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

void b64_encode(const std::string& in, std::string* out) {
    size_t i = 0;
    const size_t n = in.size();
    const uint8_t* s = (const uint8_t*)in.data();
    for (; i + 3 <= n; i += 3) {
        const uint32_t v = (uint32_t)s[i] << 16 | (uint32_t)s[i + 1] << 8 | s[i + 2];
        out->push_back(kB64[v >> 18]);
        out->push_back(kB64[(v >> 12) & 63]);
        out->push_back(kB64[(v >> 6) & 63]);
        out->push_back(kB64[v & 63]);
    }
    if (n - i == 1) {
        const uint32_t v = (uint32_t)s[i] << 16;
        out->push_back(kB64[v >> 18]);
        out->push_back(kB64[(v >> 12) & 63]);
        out->append("==");
    } else if (n - i == 2) {
        const uint32_t v = (uint32_t)s[i] << 16 | (uint32_t)s[i + 1] << 8;
        out->push_back(kB64[v >> 18]);
        out->push_back(kB64[(v >> 12) & 63]);
        out->push_back(kB64[(v >> 6) & 63]);
        out->push_back('=');
    }
}

int b64_val(char c) {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '+') return 62;
    if (c == '/') return 63;
    return -1;
}

// base64.StdEncoding.Decode as encoding/json uses it for []byte: padded, and
// '\r' / '\n' are ignored.
bool b64_decode(const std::string& in, std::string* out) {
    std::string s;
    for (char c : in)
        if (c != '\r' && c != '\n') s.push_back(c);
    if (s.size() % 4) return false;
    out->clear();
    for (size_t i = 0; i < s.size(); i += 4) {
        int v[4];
        int pad = 0;
        for (int k = 0; k < 4; ++k) {
            if (s[i + k] == '=') {
                if (i + 4 != s.size() || k < 2) return false;
                v[k] = 0;
                ++pad;
            } else {
                if (pad) return false;
                v[k] = b64_val(s[i + k]);
                if (v[k] < 0) return false;
            }
        }
        const uint32_t w = (uint32_t)v[0] << 18 | (uint32_t)v[1] << 12 | (uint32_t)v[2] << 6 | (uint32_t)v[3];
        out->push_back((char)(w >> 16));
        if (pad < 2) out->push_back((char)((w >> 8) & 0xFF));
        if (pad < 1) out->push_back((char)(w & 0xFF));
    }
    return true;
}

std::string marshal(const Wire& m) {
    std::string s = "{\"Type\":" + std::to_string(m.type) + ",\"ConnID\":" + std::to_string(m.conn) +
                    ",\"SeqNum\":" + std::to_string(m.seq) + ",\"Size\":" + std::to_string(m.size) + ",\"Payload\":";
    if (!m.has_payload) {
        s += "null";
    } else {
        s.push_back('"');
        b64_encode(m.payload, &s);
        s.push_back('"');
    }
    s.push_back('}');
    return s;
}

struct JsonIn {
    const char* s;
    size_t n, i = 0;
    void ws() {
        while (i < n && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
    }
    bool eat(char c) {
        ws();
        if (i < n && s[i] == c) {
            ++i;
            return true;
        }
        return false;
    }
    bool str(std::string* out) {  // JSON string; \u escapes kept only for ASCII (keys, base64)
        ws();
        if (i >= n || s[i] != '"') return false;
        ++i;
        out->clear();
        while (i < n && s[i] != '"') {
            if (s[i] == '\\') {
                if (i + 1 >= n) return false;
                const char e = s[i + 1];
                i += 2;
                switch (e) {
                    case '"': out->push_back('"'); break;
                    case '\\': out->push_back('\\'); break;
                    case '/': out->push_back('/'); break;
                    case 'b': out->push_back('\b'); break;
                    case 'f': out->push_back('\f'); break;
                    case 'n': out->push_back('\n'); break;
                    case 'r': out->push_back('\r'); break;
                    case 't': out->push_back('\t'); break;
                    case 'u': {
                        if (i + 4 > n) return false;
                        unsigned v = 0;
                        for (int k = 0; k < 4; ++k) {
                            const char c = s[i + k];
                            v <<= 4;
                            if (c >= '0' && c <= '9') v |= c - '0';
                            else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
                            else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
                            else return false;
                        }
                        i += 4;
                        out->push_back(v < 0x80 ? (char)v : '?');
                        break;
                    }
                    default: return false;
                }
            } else {
                out->push_back(s[i++]);
            }
        }
        if (i >= n) return false;
        ++i;
        return true;
    }
    bool integer(int64_t* v) {  // a JSON number that is an integer (Go int field)
        ws();
        const size_t b = i;
        if (i < n && s[i] == '-') ++i;
        if (i >= n || s[i] < '0' || s[i] > '9') return false;
        while (i < n && s[i] >= '0' && s[i] <= '9') ++i;
        if (i < n && (s[i] == '.' || s[i] == 'e' || s[i] == 'E')) return false;
        errno = 0;
        const std::string t(s + b, i - b);
        char* end = nullptr;
        const long long x = strtoll(t.c_str(), &end, 10);
        if (errno == ERANGE) return false;
        *v = x;
        return true;
    }
    bool lit(const char* w) {
        ws();
        const size_t k = strlen(w);
        if (i + k <= n && !memcmp(s + i, w, k)) {
            i += k;
            return true;
        }
        return false;
    }
    bool skip(int depth = 0) {  // any JSON value
        if (depth > 32) return false;
        ws();
        if (i >= n) return false;
        std::string tmp;
        int64_t x;
        if (s[i] == '"') return str(&tmp);
        if (s[i] == '{' || s[i] == '[') {
            const char close = s[i] == '{' ? '}' : ']';
            const bool obj = s[i] == '{';
            ++i;
            if (eat(close)) return true;
            do {
                if (obj && (!str(&tmp) || !eat(':'))) return false;
                if (!skip(depth + 1)) return false;
            } while (eat(','));
            return eat(close);
        }
        if (lit("null") || lit("true") || lit("false")) return true;
        if (integer(&x)) return true;
        // a non-integer number
        while (i < n && (strchr("+-.eE", s[i]) || (s[i] >= '0' && s[i] <= '9'))) ++i;
        return true;
    }
};

bool ieq(const std::string& a, const char* b) {
    if (a.size() != strlen(b)) return false;
    for (size_t k = 0; k < a.size(); ++k)
        if (tolower((unsigned char)a[k]) != tolower((unsigned char)b[k])) return false;
    return true;
}

// json.Unmarshal(buf, &lsp.Message): keys match case-insensitively, unknown
// keys are ignored, a missing field stays zero.
bool unmarshal(const char* js, size_t len, Wire* m) {
    JsonIn p{js, len};
    *m = Wire{};
    if (!p.eat('{')) return false;
    if (!p.eat('}')) {
        do {
            std::string key;
            if (!p.str(&key) || !p.eat(':')) return false;
            int64_t v = 0;
            if (ieq(key, "Type") || ieq(key, "ConnID") || ieq(key, "SeqNum") || ieq(key, "Size")) {
                if (p.lit("null")) continue;
                if (!p.integer(&v)) return false;
                if (ieq(key, "Type")) m->type = (int)v;
                else if (ieq(key, "ConnID")) m->conn = v;
                else if (ieq(key, "SeqNum")) m->seq = v;
                else m->size = v;
            } else if (ieq(key, "Payload")) {
                if (p.lit("null")) {
                    m->has_payload = false;
                    m->payload.clear();
                    continue;
                }
                std::string b;
                if (!p.str(&b) || !b64_decode(b, &m->payload)) return false;
                m->has_payload = true;
            } else if (!p.skip()) {
                return false;
            }
        } while (p.eat(','));
        if (!p.eat('}')) return false;
    }
    p.ws();
    return p.i == p.n;
}

// ---- fault injection (lspnet/staff.go) ---------------------------------
std::atomic<int> g_drop[4] = {{0}, {0}, {0}, {0}};  // client read, client write, server read, server write
std::atomic<int> g_shorten{0}, g_lengthen{0};

bool sometimes(int pct) {
    if (pct <= 0) return false;
    thread_local std::mt19937 rng{std::random_device{}()};
    return (int)(rng() % 100) < pct;
}

// ---- endpoint ------------------------------------------------------------
using Clock = std::chrono::steady_clock;

struct Conn {
    int id = 0;
    sockaddr_in addr{};
    bool connected = false;  // client: Ack(connID, 0) seen
    // sending
    int64_t next_seq = 1;
    std::deque<std::pair<int64_t, std::string>> unsent;  // window full
    std::map<int64_t, std::string> inflight;             // seq -> payload, sent, unacked
    // receiving
    int64_t expect = 1;
    std::map<int64_t, std::string> ooo;
    bool got_data = false;
    int idle = 0;  // epochs since the peer was last heard
    bool closing = false, done = false, lost = false;
    bool lost_while_closing = false;  // lost with messages still unacked during Close
    bool drained() const { return unsent.empty() && inflight.empty(); }
};

struct Event {
    int conn;
    std::string payload;
    int rc;
};

class Endpoint {
   public:
    Endpoint(bool server, const lsp_params& p) : server_(server), p_(p) {}
    ~Endpoint() {
        if (fd_ >= 0) ::close(fd_);
        if (wake_ >= 0) ::close(wake_);
    }

    int open_server(int port) {
        fd_ = ::socket(AF_INET, SOCK_DGRAM | SOCK_CLOEXEC, 0);
        if (fd_ < 0) return LSP_ESOCK;
        sockaddr_in a{};
        a.sin_family = AF_INET;
        a.sin_addr.s_addr = htonl(INADDR_ANY);
        a.sin_port = htons((uint16_t)port);
        if (::bind(fd_, (sockaddr*)&a, sizeof a) != 0) return LSP_ESOCK;
        socklen_t l = sizeof a;
        ::getsockname(fd_, (sockaddr*)&a, &l);
        port_ = ntohs(a.sin_port);
        return start();
    }

    int open_client(const char* hostport) {
        std::string hp(hostport ? hostport : "");
        const size_t c = hp.rfind(':');
        if (c == std::string::npos) return LSP_ESOCK;
        std::string host = hp.substr(0, c), port = hp.substr(c + 1);
        if (host.empty()) host = "127.0.0.1";
        if (host.size() > 2 && host.front() == '[') return LSP_ESOCK;  // IPv6 literal: not served
        addrinfo hints{}, *res = nullptr;
        hints.ai_family = AF_INET;
        hints.ai_socktype = SOCK_DGRAM;
        if (::getaddrinfo(host.c_str(), port.c_str(), &hints, &res) != 0 || !res) return LSP_ESOCK;
        memcpy(&cli_.addr, res->ai_addr, sizeof(sockaddr_in));
        ::freeaddrinfo(res);
        fd_ = ::socket(AF_INET, SOCK_DGRAM | SOCK_CLOEXEC, 0);
        if (fd_ < 0) return LSP_ESOCK;
        if (::connect(fd_, (sockaddr*)&cli_.addr, sizeof cli_.addr) != 0) return LSP_ESOCK;  // DialUDP
        int rc = start();
        if (rc) return rc;
        std::unique_lock<std::mutex> lk(mu_);
        send_ctl(cli_, kConnect, 0, 0);
        cv_.wait(lk, [&] { return cli_.connected || connect_failed_; });
        if (!cli_.connected) {
            lk.unlock();
            stop();
            return LSP_ECONNECT;
        }
        return LSP_OK;
    }

    int port() const { return port_; }
    int conn_id() {
        std::lock_guard<std::mutex> lk(mu_);
        return cli_.id;
    }

    // Read: server and client.  Error events are sticky on the client.
    int read(int* conn, uint8_t* buf, size_t cap, size_t* len, int timeout_ms) {
        std::unique_lock<std::mutex> lk(mu_);
        ++readers_;
        auto ready = [&] { return !events_.empty() || stopping_ || (!server_ && sticky_ != LSP_OK); };
        bool ok = true;
        if (timeout_ms < 0)
            cv_.wait(lk, ready);
        else
            // system_clock: pthread_cond_timedwait, which ThreadSanitizer
            // intercepts (GCC 11's TSan misses pthread_cond_clockwait, the
            // steady-clock wait, and then reports false double locks)
            ok = cv_.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(timeout_ms), ready);
        int rc;
        if (!events_.empty()) {
            Event& e = events_.front();
            if (conn) *conn = e.conn;
            if (len) *len = e.payload.size();
            if (e.rc == LSP_OK && e.payload.size() > cap) {
                rc = LSP_ESHORT;  // stays queued
            } else {
                if (e.rc == LSP_OK && !e.payload.empty()) memcpy(buf, e.payload.data(), e.payload.size());
                rc = e.rc;
                if (!server_ && rc != LSP_OK) sticky_ = rc;
                if (server_ && rc != LSP_OK) forget(e.conn, rc);  // the caller now knows: free the Conn
                events_.pop_front();
            }
        } else if (!server_ && sticky_ != LSP_OK) {
            rc = sticky_;
        } else if (stopping_) {
            if (conn) *conn = 0;
            rc = LSP_ECLOSED;
        } else {
            rc = ok ? LSP_ECLOSED : LSP_ETIMEOUT;
        }
        if (--readers_ == 0) cv_.notify_all();
        return rc;
    }

    int write(int conn, const uint8_t* p, size_t n) {
        std::lock_guard<std::mutex> lk(mu_);
        Conn* c = nullptr;
        if (server_) {
            auto it = conns_.find(conn);
            if (it == conns_.end()) {
                auto g = gone_.find(conn);
                return g == gone_.end() ? LSP_EINVAL : g->second;
            }
            c = &it->second;
            if (closing_all_) return LSP_ECLOSED;
        } else {
            c = &cli_;
        }
        if (c->lost) return LSP_ELOST;
        if (c->done || c->closing) return LSP_ECLOSED;
        if (frame_size(*c, n) > kMaxDatagram) return LSP_ETOOBIG;  // could never be delivered
        c->unsent.emplace_back(c->next_seq++, std::string((const char*)p, n));
        pump(*c);
        return LSP_OK;
    }

    int close_conn(int conn) {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = conns_.find(conn);
        if (it == conns_.end()) return gone_.count(conn) ? LSP_ECLOSED : LSP_EINVAL;
        if (it->second.done) return LSP_EINVAL;
        it->second.closing = true;
        maybe_finish(it->second);
        return LSP_OK;
    }

    // Client.Close / Server.Close: wait until everything written is acked or
    // its peer is lost, then stop the thread.
    int close_all() {
        int rc = LSP_OK;
        {
            std::unique_lock<std::mutex> lk(mu_);
            if (server_) {
                closing_all_ = true;
                for (auto& kv : conns_) kv.second.closing = true;
                cv_.wait(lk, [&] {
                    for (auto& kv : conns_)
                        if (!kv.second.done && !kv.second.drained()) return false;
                    return true;
                });
                if (lost_unacked_) rc = LSP_ELOST;  // already forgotten ones (forget)
                for (auto& kv : conns_)
                    if (kv.second.lost && kv.second.lost_while_closing) rc = LSP_ELOST;
            } else {
                cli_.closing = true;
                cv_.wait(lk, [&] { return cli_.drained() || cli_.lost; });
                if (cli_.lost && !cli_.drained()) rc = LSP_ELOST;
            }
        }
        stop();
        return rc;
    }

    void stop() {
        {
            std::unique_lock<std::mutex> lk(mu_);
            stopping_ = true;
            cv_.notify_all();
            cv_.wait(lk, [&] { return readers_ == 0; });
        }
        wake();
        if (th_.joinable()) th_.join();
    }

   private:
    bool server_;
    lsp_params p_;
    int fd_ = -1, wake_ = -1, port_ = 0;
    std::thread th_;
    std::mutex mu_;
    std::condition_variable cv_;
    bool stopping_ = false, connect_failed_ = false, closing_all_ = false;
    int readers_ = 0;
    int sticky_ = LSP_OK;
    std::deque<Event> events_;
    Conn cli_;                   // client side: the one connection
    std::map<int, Conn> conns_;  // server side, by connID
    std::map<int, int> gone_;    // server side: connIDs whose end Read reported -> LSP_ELOST / LSP_ECLOSED
    bool lost_unacked_ = false;  // server side: a forgotten conn was lost while closing with data unacked
    std::map<uint64_t, int> by_addr_;
    int next_id_ = 1;

    static uint64_t addr_key(const sockaddr_in& a) {
        return (uint64_t)ntohl(a.sin_addr.s_addr) << 16 | ntohs(a.sin_port);
    }

    int start() {
        wake_ = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
        if (wake_ < 0) return LSP_ESOCK;
        th_ = std::thread([this] { loop(); });
        return LSP_OK;
    }
    void wake() {
        const uint64_t one = 1;
        if (wake_ >= 0) (void)!::write(wake_, &one, sizeof one);
    }

    // Bytes of the Data datagram that would carry an n-byte payload on c.
    size_t frame_size(const Conn& c, size_t n) const {
        Wire w;
        w.type = kData;
        w.conn = c.id;
        w.seq = c.next_seq;
        w.size = (int64_t)n;
        w.has_payload = true;
        w.payload.assign(n, '\0');
        return marshal(w).size();
    }

    // A server connection whose terminal event the caller has read: drop its
    // buffers, remember only how it ended (for later write / close_conn), and
    // whether it was lost with messages unacked while closing (for Close).
    // Only the last kGoneCap ended connIDs are remembered (ids only grow, so
    // the smallest go first): a long-running server seeing many short client
    // connections stays bounded, and a write to a long-forgotten id gets
    // LSP_EINVAL instead of its old LSP_ELOST / LSP_ECLOSED.
    static constexpr size_t kGoneCap = 1u << 16;
    void forget(int id, int rc) {
        auto it = conns_.find(id);
        if (it == conns_.end() || !it->second.done) return;
        if (it->second.lost && it->second.lost_while_closing) lost_unacked_ = true;
        gone_[id] = rc;
        conns_.erase(it);
        while (gone_.size() > kGoneCap) gone_.erase(gone_.begin());
    }

    // -- datagrams out (mu_ held) --
    void send_wire(const Conn& c, const Wire& m) {
        if (sometimes(g_drop[server_ ? 3 : 1].load())) return;
        Wire w = m;
        if (w.type == kData) {  // lspnet's payload mangling, Size unchanged
            if (sometimes(g_shorten.load())) w.payload.resize(w.payload.size() / 2);
            else if (sometimes(g_lengthen.load())) w.payload.append(w.payload.size() + 1, 'x');
        }
        const std::string b = marshal(w);
        if (server_)
            (void)::sendto(fd_, b.data(), b.size(), MSG_DONTWAIT, (const sockaddr*)&c.addr, sizeof c.addr);
        else
            (void)::send(fd_, b.data(), b.size(), MSG_DONTWAIT);
    }
    void send_ctl(const Conn& c, int type, int64_t conn, int64_t seq) {
        Wire w;
        w.type = type;
        w.conn = conn;
        w.seq = seq;
        send_wire(c, w);
    }
    void send_data(const Conn& c, int64_t seq, const std::string& payload) {
        Wire w;
        w.type = kData;
        w.conn = c.id;
        w.seq = seq;
        w.size = (int64_t)payload.size();
        w.has_payload = true;
        w.payload = payload;
        send_wire(c, w);
    }
    // Sliding window: Data seq may be in flight only while seq < oldest unacked + WindowSize.
    void pump(Conn& c) {
        if (!c.connected && !server_) return;
        while (!c.unsent.empty()) {
            const int64_t oldest = c.inflight.empty() ? c.unsent.front().first : c.inflight.begin()->first;
            auto& f = c.unsent.front();
            if (f.first >= oldest + p_.window_size) break;
            send_data(c, f.first, f.second);
            c.inflight.emplace(f.first, std::move(f.second));
            c.unsent.pop_front();
        }
    }
    void maybe_finish(Conn& c) {  // server: a closing connection whose messages are all acked
        if (server_ && c.closing && !c.done && c.drained()) {
            c.done = true;
            by_addr_.erase(addr_key(c.addr));
            if (!closing_all_) events_.push_back(Event{c.id, std::string(), LSP_ECLOSED});
        }
        cv_.notify_all();
    }
    void mark_lost(Conn& c) {
        c.lost = true;
        if (c.closing) c.lost_while_closing = !c.drained();
        c.done = true;
        if (server_) by_addr_.erase(addr_key(c.addr));
        events_.push_back(Event{c.id, std::string(), LSP_ELOST});
        cv_.notify_all();
    }

    // -- datagrams in (mu_ held) --
    void on_data(Conn& c, Wire& m) {
        if (!m.has_payload) m.payload.clear();
        if (m.size < 0 || (int64_t)m.payload.size() < m.size) return;  // short: dropped, not acked
        if ((int64_t)m.payload.size() > m.size) m.payload.resize((size_t)m.size);
        send_ctl(c, kAck, c.id, m.seq);
        if (m.seq >= c.expect && !c.ooo.count(m.seq)) {
            c.ooo.emplace(m.seq, std::move(m.payload));
            for (auto it = c.ooo.find(c.expect); it != c.ooo.end(); it = c.ooo.find(c.expect)) {
                if (!c.done) events_.push_back(Event{c.id, std::move(it->second), LSP_OK});
                c.ooo.erase(it);
                ++c.expect;
            }
            cv_.notify_all();
        }
        c.got_data = true;
    }
    void on_ack(Conn& c, const Wire& m) {
        if (m.seq == 0) return;  // heartbeat / connect ack
        if (c.inflight.erase(m.seq)) {
            pump(c);
            maybe_finish(c);
            cv_.notify_all();
        }
    }

    void on_datagram(const char* b, size_t n, const sockaddr_in& from) {
        if (sometimes(g_drop[server_ ? 2 : 0].load())) return;
        Wire m;
        if (!unmarshal(b, n, &m)) return;
        std::lock_guard<std::mutex> lk(mu_);
        if (stopping_) return;
        if (server_) {
            if (m.type == kConnect) {
                auto a = by_addr_.find(addr_key(from));
                if (a != by_addr_.end()) {  // a resent Connect: ack it again
                    send_ctl(conns_[a->second], kAck, a->second, 0);
                    return;
                }
                if (closing_all_) return;
                const int id = next_id_++;
                Conn& c = conns_[id];
                c.id = id;
                c.addr = from;
                c.connected = true;
                by_addr_[addr_key(from)] = id;
                send_ctl(c, kAck, id, 0);
                return;
            }
            auto it = conns_.find((int)m.conn);
            if (it == conns_.end() || it->second.done || addr_key(it->second.addr) != addr_key(from)) return;
            Conn& c = it->second;
            c.idle = 0;
            if (m.type == kData) on_data(c, m);
            else if (m.type == kAck) on_ack(c, m);
            return;
        }
        if (cli_.done) return;
        if (!cli_.connected) {
            if ((m.type == kAck && m.seq == 0) || m.type == kData) {  // a Data implies the Ack was lost
                cli_.connected = true;
                cli_.id = (int)m.conn;
                cv_.notify_all();
            } else {
                return;
            }
        }
        if (m.conn != cli_.id) return;
        cli_.idle = 0;
        if (m.type == kData) on_data(cli_, m);
        else if (m.type == kAck) on_ack(cli_, m);
    }

    void epoch_conn(Conn& c) {
        if (c.done) return;
        if (++c.idle > p_.epoch_limit) {
            mark_lost(c);
            return;
        }
        for (auto& kv : c.inflight) send_data(c, kv.first, kv.second);
        if (!c.got_data) {
            send_ctl(c, kAck, c.id, 0);
        } else {
            for (int64_t k = 1; k <= p_.window_size && c.expect - k >= 1; ++k) send_ctl(c, kAck, c.id, c.expect - k);
        }
    }

    void epoch() {
        std::lock_guard<std::mutex> lk(mu_);
        if (stopping_) return;
        if (server_) {
            for (auto& kv : conns_) epoch_conn(kv.second);
            return;
        }
        if (!cli_.connected) {
            if (++cli_.idle > p_.epoch_limit) {
                connect_failed_ = true;
                cv_.notify_all();
            } else {
                send_ctl(cli_, kConnect, 0, 0);
            }
            return;
        }
        epoch_conn(cli_);
    }

    void loop() {
        const auto period = std::chrono::milliseconds(std::max(1, p_.epoch_millis));
        auto next = Clock::now() + period;
        std::vector<char> buf(65536);
        for (;;) {
            {
                std::lock_guard<std::mutex> lk(mu_);
                if (stopping_) return;
            }
            const auto now = Clock::now();
            int ms = 0;
            if (next > now) ms = (int)std::chrono::duration_cast<std::chrono::milliseconds>(next - now).count() + 1;
            pollfd pf[2] = {{fd_, POLLIN, 0}, {wake_, POLLIN, 0}};
            ::poll(pf, 2, ms);
            if (pf[1].revents & POLLIN) {
                uint64_t v;
                (void)!::read(wake_, &v, sizeof v);
            }
            if (pf[0].revents & POLLIN) {
                for (;;) {
                    sockaddr_in from{};
                    socklen_t fl = sizeof from;
                    const ssize_t k = ::recvfrom(fd_, buf.data(), buf.size(), MSG_DONTWAIT, (sockaddr*)&from, &fl);
                    if (k < 0) break;  // EAGAIN, or ECONNREFUSED from an ICMP error: nothing to read
                    on_datagram(buf.data(), (size_t)k, from);
                }
            }
            if (Clock::now() >= next) {
                epoch();
                next += period;
                if (next < Clock::now()) next = Clock::now() + period;
            }
        }
    }
};

}  // namespace
}  // namespace lsp440

using lsp440::Endpoint;

struct lsp_client {
    Endpoint* ep;
};
struct lsp_server {
    Endpoint* ep;
};

namespace {
lsp_params params_or_default(const lsp_params* p) {
    lsp_params d;
    lsp_default_params(&d);
    if (!p) return d;
    lsp_params q = *p;
    if (q.epoch_limit < 1) q.epoch_limit = d.epoch_limit;
    if (q.epoch_millis < 1) q.epoch_millis = d.epoch_millis;
    if (q.window_size < 1) q.window_size = d.window_size;
    return q;
}
}  // namespace

extern "C" {

void lsp_default_params(lsp_params* p) {
    if (!p) return;
    p->epoch_limit = 5;
    p->epoch_millis = 2000;
    p->window_size = 1;
}

int lsp_client_new(const char* hostport, const lsp_params* params, lsp_client** out) {
    if (!out) return LSP_EINVAL;
    *out = nullptr;
    auto* ep = new Endpoint(false, params_or_default(params));
    const int rc = ep->open_client(hostport);
    if (rc != LSP_OK) {
        ep->stop();
        delete ep;
        return rc;
    }
    *out = new lsp_client{ep};
    return LSP_OK;
}

int lsp_client_conn_id(lsp_client* c) { return c ? c->ep->conn_id() : LSP_EINVAL; }

int lsp_client_read(lsp_client* c, uint8_t* buf, size_t cap, size_t* len, int timeout_ms) {
    if (!c || (!buf && cap)) return LSP_EINVAL;
    return c->ep->read(nullptr, buf, cap, len, timeout_ms);
}

int lsp_client_write(lsp_client* c, const uint8_t* payload, size_t len) {
    if (!c || (!payload && len)) return LSP_EINVAL;
    return c->ep->write(0, payload, len);
}

int lsp_client_close(lsp_client* c) {
    if (!c) return LSP_EINVAL;
    const int rc = c->ep->close_all();
    delete c->ep;
    delete c;
    return rc;
}

int lsp_server_new(int port, const lsp_params* params, lsp_server** out) {
    if (!out || port < 0 || port > 65535) return LSP_EINVAL;
    *out = nullptr;
    auto* ep = new Endpoint(true, params_or_default(params));
    const int rc = ep->open_server(port);
    if (rc != LSP_OK) {
        ep->stop();
        delete ep;
        return rc;
    }
    *out = new lsp_server{ep};
    return LSP_OK;
}

int lsp_server_port(lsp_server* s) { return s ? s->ep->port() : LSP_EINVAL; }

int lsp_server_read(lsp_server* s, int* conn_id, uint8_t* buf, size_t cap, size_t* len, int timeout_ms) {
    if (!s || (!buf && cap)) return LSP_EINVAL;
    return s->ep->read(conn_id, buf, cap, len, timeout_ms);
}

int lsp_server_write(lsp_server* s, int conn_id, const uint8_t* payload, size_t len) {
    if (!s || (!payload && len)) return LSP_EINVAL;
    return s->ep->write(conn_id, payload, len);
}

int lsp_server_close_conn(lsp_server* s, int conn_id) { return s ? s->ep->close_conn(conn_id) : LSP_EINVAL; }

int lsp_server_close(lsp_server* s) {
    if (!s) return LSP_EINVAL;
    const int rc = s->ep->close_all();
    delete s->ep;
    delete s;
    return rc;
}

void lsp_set_drop_percent(int client_read, int client_write, int server_read, int server_write) {
    lsp440::g_drop[0] = client_read;
    lsp440::g_drop[1] = client_write;
    lsp440::g_drop[2] = server_read;
    lsp440::g_drop[3] = server_write;
}

void lsp_set_msg_mangle_percent(int shorten, int lengthen) {
    lsp440::g_shorten = shorten;
    lsp440::g_lengthen = lengthen;
}

int lsp_marshal(int type, int64_t conn_id, int64_t seq, int64_t size, const uint8_t* payload, size_t plen,
                int has_payload, char* out, size_t cap, size_t* len) {
    if ((!payload && plen) || (!out && cap)) return LSP_EINVAL;
    lsp440::Wire w;
    w.type = type;
    w.conn = conn_id;
    w.seq = seq;
    w.size = size;
    w.has_payload = has_payload != 0;
    if (w.has_payload && plen) w.payload.assign((const char*)payload, plen);
    const std::string s = lsp440::marshal(w);
    if (len) *len = s.size();
    if (s.size() > cap) return LSP_ESHORT;
    memcpy(out, s.data(), s.size());
    return LSP_OK;
}

int lsp_unmarshal(const char* js, size_t jlen, int* type, int64_t* conn_id, int64_t* seq, int64_t* size,
                  uint8_t* payload, size_t cap, size_t* plen, int* has_payload) {
    if (!js && jlen) return LSP_EINVAL;
    lsp440::Wire w;
    if (!lsp440::unmarshal(js, jlen, &w)) return LSP_EINVAL;
    if (type) *type = w.type;
    if (conn_id) *conn_id = w.conn;
    if (seq) *seq = w.seq;
    if (size) *size = w.size;
    if (has_payload) *has_payload = w.has_payload;
    if (plen) *plen = w.payload.size();
    if (w.payload.size() > cap) return LSP_ESHORT;
    if (!w.payload.empty()) memcpy(payload, w.payload.data(), w.payload.size());
    return LSP_OK;
}

}  // extern "C"
