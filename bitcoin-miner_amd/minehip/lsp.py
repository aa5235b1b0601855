"""ctypes face of liblsp440.so (include/lsp440.h): the LSP transport, named
after the reference's Go API so tests read like lsp/*_test.go.

  NewParams()                      lsp/params.go:34-40
  NewClient(hostport, params)      lsp/client_impl.go:56 (Client: client_api.go:6-30)
  NewServer(port, params)          lsp/server_impl.go:35 (Server: server_api.go:6-39)
  set_drop_percent / set_msg_mangle_percent
                                   lspnet/staff.go fault injection (tests)
  marshal / unmarshal              lsp/util.go:19-33 (one datagram)

Read / Write / Close return errors Go-style: Read() -> (payload, err), where
err is None or an LspError.  Blocking calls release the GIL (ctypes).
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liblsp440.so")

LSP_OK = 0
LSP_ECLOSED = -10
LSP_ELOST = -11
LSP_ECONNECT = -12
LSP_ETIMEOUT = -13
LSP_EINVAL = -14
LSP_ESOCK = -15
LSP_ESHORT = -16
LSP_ETOOBIG = -17
MAX_DATAGRAM = 65507  # LSP_MAX_DATAGRAM (include/lsp440.h)

MsgConnect, MsgData, MsgAck = 0, 1, 2  # lsp/message.go:10-14

#: every symbol include/lsp440.h declares
EXPORTS = (
    "lsp_default_params", "lsp_client_new", "lsp_client_conn_id", "lsp_client_read", "lsp_client_write",
    "lsp_client_close", "lsp_server_new", "lsp_server_port", "lsp_server_read", "lsp_server_write",
    "lsp_server_close_conn", "lsp_server_close", "lsp_set_drop_percent", "lsp_set_msg_mangle_percent",
    "lsp_marshal", "lsp_unmarshal",
)


class lsp_params(ctypes.Structure):
    _fields_ = [("epoch_limit", ctypes.c_int), ("epoch_millis", ctypes.c_int), ("window_size", ctypes.c_int)]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run `make` at the repository root")
    L = ctypes.CDLL(LIB_PATH)
    P, I, SZ = ctypes.POINTER, ctypes.c_int, ctypes.c_size_t
    vp, u8p, i64 = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64
    L.lsp_default_params.argtypes = [P(lsp_params)]
    L.lsp_default_params.restype = None
    L.lsp_client_new.argtypes = [ctypes.c_char_p, P(lsp_params), P(vp)]
    L.lsp_client_conn_id.argtypes = [vp]
    L.lsp_client_read.argtypes = [vp, u8p, SZ, P(SZ), I]
    L.lsp_client_write.argtypes = [vp, u8p, SZ]
    L.lsp_client_close.argtypes = [vp]
    L.lsp_server_new.argtypes = [I, P(lsp_params), P(vp)]
    L.lsp_server_port.argtypes = [vp]
    L.lsp_server_read.argtypes = [vp, P(I), u8p, SZ, P(SZ), I]
    L.lsp_server_write.argtypes = [vp, I, u8p, SZ]
    L.lsp_server_close_conn.argtypes = [vp, I]
    L.lsp_server_close.argtypes = [vp]
    L.lsp_set_drop_percent.argtypes = [I, I, I, I]
    L.lsp_set_drop_percent.restype = None
    L.lsp_set_msg_mangle_percent.argtypes = [I, I]
    L.lsp_set_msg_mangle_percent.restype = None
    L.lsp_marshal.argtypes = [I, i64, i64, i64, u8p, SZ, I, ctypes.c_char_p, SZ, P(SZ)]
    L.lsp_unmarshal.argtypes = [ctypes.c_char_p, SZ, P(I), P(i64), P(i64), P(i64), u8p, SZ, P(SZ), P(I)]
    return L


lib = _load()

_NAMES = {LSP_ECLOSED: "connection closed", LSP_ELOST: "connection lost",
          LSP_ECONNECT: "can not establish connection", LSP_ETIMEOUT: "timeout",
          LSP_EINVAL: "invalid argument", LSP_ESOCK: "socket error", LSP_ESHORT: "buffer too small",
          LSP_ETOOBIG: "message too big for one datagram"}


class LspError(Exception):
    def __init__(self, code):
        super().__init__(_NAMES.get(code, f"lsp error {code}"))
        self.code = code


def _err(rc):
    return None if rc == LSP_OK else LspError(rc)


def NewParams(epoch_limit=None, epoch_millis=None, window_size=None):  # noqa: N802
    p = lsp_params()
    lib.lsp_default_params(ctypes.byref(p))
    if epoch_limit is not None:
        p.epoch_limit = epoch_limit
    if epoch_millis is not None:
        p.epoch_millis = epoch_millis
    if window_size is not None:
        p.window_size = window_size
    return p


def Params(epoch_limit, epoch_millis, window_size):  # noqa: N802  (&Params{EpochLimit, EpochMillis, WindowSize})
    return lsp_params(epoch_limit, epoch_millis, window_size)


class Client:
    """lsp.Client (client_api.go:6-30)."""

    def __init__(self, h):
        self._h = h
        self._buf = ctypes.create_string_buffer(1 << 16)

    def ConnID(self):  # noqa: N802
        return lib.lsp_client_conn_id(self._h)

    def Read(self, timeout_ms=-1):  # noqa: N802
        n = ctypes.c_size_t()
        while True:
            rc = lib.lsp_client_read(self._h, self._buf, len(self._buf), ctypes.byref(n), timeout_ms)
            if rc != LSP_ESHORT:
                break
            self._buf = ctypes.create_string_buffer(n.value)
        return (self._buf.raw[:n.value] if rc == LSP_OK else None), _err(rc)

    def Write(self, payload):  # noqa: N802
        return _err(lib.lsp_client_write(self._h, bytes(payload), len(payload)))

    def Close(self):  # noqa: N802
        h, self._h = self._h, None
        return _err(lib.lsp_client_close(h)) if h else None


class Server:
    """lsp.Server (server_api.go:6-39)."""

    def __init__(self, h):
        self._h = h
        self._buf = ctypes.create_string_buffer(1 << 16)

    @property
    def port(self):
        return lib.lsp_server_port(self._h)

    def Read(self, timeout_ms=-1):  # noqa: N802
        conn, n = ctypes.c_int(), ctypes.c_size_t()
        while True:
            rc = lib.lsp_server_read(self._h, ctypes.byref(conn), self._buf, len(self._buf), ctypes.byref(n),
                                     timeout_ms)
            if rc != LSP_ESHORT:
                break
            self._buf = ctypes.create_string_buffer(n.value)
        return conn.value, (self._buf.raw[:n.value] if rc == LSP_OK else None), _err(rc)

    def Write(self, conn_id, payload):  # noqa: N802
        return _err(lib.lsp_server_write(self._h, conn_id, bytes(payload), len(payload)))

    def CloseConn(self, conn_id):  # noqa: N802
        return _err(lib.lsp_server_close_conn(self._h, conn_id))

    def Close(self):  # noqa: N802
        h, self._h = self._h, None
        return _err(lib.lsp_server_close(h)) if h else None


def NewClient(hostport, params=None):  # noqa: N802
    h = ctypes.c_void_p()
    rc = lib.lsp_client_new(hostport.encode(), ctypes.byref(params) if params is not None else None,
                            ctypes.byref(h))
    return (Client(h) if rc == LSP_OK else None), _err(rc)


def NewServer(port, params=None):  # noqa: N802
    h = ctypes.c_void_p()
    rc = lib.lsp_server_new(port, ctypes.byref(params) if params is not None else None, ctypes.byref(h))
    return (Server(h) if rc == LSP_OK else None), _err(rc)


def set_drop_percent(client_read=0, client_write=0, server_read=0, server_write=0):
    lib.lsp_set_drop_percent(client_read, client_write, server_read, server_write)


def set_msg_mangle_percent(shorten=0, lengthen=0):
    lib.lsp_set_msg_mangle_percent(shorten, lengthen)


def marshal(type_, conn_id=0, seq=0, size=0, payload=None):
    """json.Marshal(&lsp.Message{...}); payload None = nil (null)."""
    out = ctypes.create_string_buffer(4096 + 2 * len(payload or b""))
    n = ctypes.c_size_t()
    p = bytes(payload) if payload is not None else None
    rc = lib.lsp_marshal(type_, conn_id, seq, size, p, len(p or b""), 1 if p is not None else 0, out, len(out),
                         ctypes.byref(n))
    if rc != LSP_OK:
        raise LspError(rc)
    return out.raw[:n.value]


def unmarshal(js):
    """json.Unmarshal into lsp.Message -> dict, or None if it is not one."""
    t, c, s, z, n, hp = ctypes.c_int(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_size_t(), \
        ctypes.c_int()
    buf = ctypes.create_string_buffer(len(js) + 1)
    rc = lib.lsp_unmarshal(js, len(js), ctypes.byref(t), ctypes.byref(c), ctypes.byref(s), ctypes.byref(z), buf,
                           len(buf), ctypes.byref(n), ctypes.byref(hp))
    if rc != LSP_OK:
        return None
    return {"Type": t.value, "ConnID": c.value, "SeqNum": s.value, "Size": z.value,
            "Payload": buf.raw[:n.value] if hp.value else None}
