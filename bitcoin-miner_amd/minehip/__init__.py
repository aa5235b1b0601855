"""minehip -- MI355X (gfx950) SHA-256 nonce search for the CMU 15-440 miner.

Python face of libminehip.so, named after the reference's own API so parity
tests read like the reference (line numbers into the reference repo):

  Hash(msg, nonce)           bitcoin/hash.go:13-17, computed on the GPU
  hash_batch(msg, nonces)    the same for many nonces
  search(msg, lower, upper)  the miner scan (stub miner.go:33)
  search_multi(...)          the scan sharded over several devices
  Message / NewRequest / NewResult / NewJoin / marshal / unmarshal
                             bitcoin/message.go:7-62 with Go encoding/json bytes
  miner_handle(request)      one miner step: Request payload -> Result payload

All compute goes through the C-ABI; there is no host fallback.
"""
import ctypes

import numpy as np

from ._lib import lib, mh_piece, mh_message, mh_kernel_stat, mh_span, OPS_PER_BLOCK, EXPORTS, LIB_PATH  # noqa: F401
from ._lib import MH_OK, MH_EINVAL, MH_ERANGE, MH_ETOOLONG, MH_ENODEV, MH_EHIP  # noqa: F401
from ._lib import MH_ENOTREQ, MH_EINTERNAL, MH_EREJECTED  # noqa: F401

U64_MAX = (1 << 64) - 1


class MinehipError(RuntimeError):
    def __init__(self, code, what):
        super().__init__(f"minehip error {code}: {what}")
        self.code = code


def _check(rc):
    if rc != MH_OK:
        raise MinehipError(rc, lib.mh_last_error().decode("utf-8", "replace"))


def _b(msg):
    return msg.encode("utf-8") if isinstance(msg, str) else bytes(msg)


def device_count():
    return lib.mh_device_count()


def search(msg, lower, upper, dev=0):
    """(hash, nonce) = lexicographic min of (Hash(msg, n), n), n in [lower, upper]."""
    m = _b(msg)
    h = ctypes.c_uint64()
    n = ctypes.c_uint64()
    _check(lib.mh_search(dev, m, len(m), lower, upper, ctypes.byref(h), ctypes.byref(n)))
    return h.value, n.value


def search_multi(msg, lower, upper, devs=None, chunk=0):
    m = _b(msg)
    if devs is None:
        devs = list(range(device_count()))
    arr = (ctypes.c_int * len(devs))(*devs)
    h = ctypes.c_uint64()
    n = ctypes.c_uint64()
    _check(lib.mh_search_multi(arr, len(devs), m, len(m), lower, upper, chunk, ctypes.byref(h),
                               ctypes.byref(n)))
    return h.value, n.value


def hash_batch(msg, nonces, dev=0):
    m = _b(msg)
    a = np.ascontiguousarray(nonces, dtype=np.uint64)
    out = np.empty_like(a)
    p = ctypes.POINTER(ctypes.c_uint64)
    _check(lib.mh_hash_batch(dev, m, len(m), a.ctypes.data_as(p), a.size, out.ctypes.data_as(p)))
    return out


def Hash(msg, nonce, dev=0):  # noqa: N802  (reference name, bitcoin/hash.go:13)
    return int(hash_batch(msg, [nonce], dev)[0])


def plan(msg, lower, upper, cap=1 << 16):
    """Host-only: the launch plan of a search (list of dicts)."""
    m = _b(msg)
    buf = (mh_piece * cap)()
    k = lib.mh_plan(m, len(m), lower, upper, buf, cap)
    if k < 0:
        _check(k)
    if k > cap:
        raise ValueError("plan longer than cap")
    return [{f: getattr(buf[i], f) for f, _ in mh_piece._fields_} for i in range(k)]


def multi_plan(msg, lower, upper, ndev, weights=None, cap=1 << 12):
    """Host-only: how search_multi (chunk = 0) splits [lower, upper] over ndev workers with rates in
    proportion to `weights` (None = equal): head shards, then tail chunks (list of dicts)."""
    if weights is not None and len(weights) != ndev:
        raise ValueError(f"multi_plan: {len(weights)} weights for {ndev} workers")
    m = _b(msg)
    buf = (mh_span * cap)()
    w = None if weights is None else (ctypes.c_double * ndev)(*weights)
    k = lib.mh_multi_plan(m, len(m), lower, upper, w, ndev, buf, cap)
    if k < 0:
        _check(k)
    if k > cap:
        raise ValueError("split longer than cap")
    return [{f: getattr(buf[i], f) for f, _ in mh_span._fields_} for i in range(k)]


def multi_rates(devs):
    """The per-process device rates search_multi sizes its shards by (cost units per ns, 0 = none)."""
    arr = (ctypes.c_int * len(devs))(*devs)
    out = (ctypes.c_double * len(devs))()
    _check(lib.mh_multi_rates(arr, len(devs), out))
    return list(out)


def profile_enable(dev=0, on=True):
    _check(lib.mh_profile_enable(dev, 1 if on else 0))


def profile_read(dev=0):
    out = (ctypes.c_uint64 * 8)()
    _check(lib.mh_profile_read(dev, out, 8))
    keys = ("fast_launches", "fast_nonces", "fast_ns", "fast_ops", "generic_nonces", "generic_ns", "fast_slots")
    return {k: int(out[i]) for i, k in enumerate(keys)}


def profile_kernels(dev=0):
    """Per fast_search<J, MODE> variant and lane length L (lo_digits): launches, nonces, ns, ops
    (largest ns first).  `name` is the kernel's name in a rocprofv3 trace (the same for every L)."""
    cap = 256
    buf = (mh_kernel_stat * cap)()
    n = lib.mh_profile_kernels(dev, buf, cap)
    if n < 0:
        _check(n)
    out = [{f: int(getattr(buf[i], f)) for f, _ in mh_kernel_stat._fields_ if f != "reserved"}
           for i in range(min(n, cap))]
    for k in out:
        k["name"] = f"mh::fast_search<{k['word']}, {k['mode']}>"
    return sorted(out, key=lambda k: -k["ns"])


# ---- bitcoin/message.go mirror --------------------------------------------
Join, Request, Result = 0, 1, 2  # MsgType iota, message.go:9-13


class Message:
    """bitcoin.Message (message.go:18-23)."""

    __slots__ = ("Type", "Data", "Lower", "Upper", "Hash", "Nonce")

    def __init__(self, Type=0, Data=b"", Lower=0, Upper=0, Hash=0, Nonce=0):  # noqa: N803
        self.Type, self.Data = Type, _b(Data)
        self.Lower, self.Upper, self.Hash, self.Nonce = Lower, Upper, Hash, Nonce

    def __eq__(self, o):
        return isinstance(o, Message) and all(getattr(self, k) == getattr(o, k) for k in self.__slots__)

    def __repr__(self):
        return self.String()

    def String(self):  # noqa: N802  (message.go:51-62)
        if self.Type == Request:
            return "[Request %s %d %d]" % (self.Data.decode("utf-8", "replace"), self.Lower, self.Upper)
        if self.Type == Result:
            return "[Result %d %d]" % (self.Hash, self.Nonce)
        if self.Type == Join:
            return "[Join]"
        return ""


def NewRequest(data, lower, upper):  # noqa: N802  (message.go:27-34)
    return Message(Request, data, lower, upper)


def NewResult(hash_, nonce):  # noqa: N802  (message.go:38-44)
    return Message(Result, b"", 0, 0, hash_, nonce)


def NewJoin():  # noqa: N802  (message.go:47-49)
    return Message(Join)


def marshal(m):
    """json.Marshal(m) as Go produces it."""
    need = ctypes.c_size_t()
    lib.mh_msg_encode(m.Type, m.Data, len(m.Data), m.Lower, m.Upper, m.Hash, m.Nonce, None, 0,
                      ctypes.byref(need))
    buf = ctypes.create_string_buffer(need.value)
    _check(lib.mh_msg_encode(m.Type, m.Data, len(m.Data), m.Lower, m.Upper, m.Hash, m.Nonce, buf,
                             need.value, ctypes.byref(need)))
    return buf.raw[:need.value]


def unmarshal(payload):
    """json.Unmarshal(payload, &m) with Go's decoding rules."""
    p = _b(payload)
    mm = mh_message()
    cap = len(p) + 16
    data = ctypes.create_string_buffer(cap)
    _check(lib.mh_msg_decode(p, len(p), ctypes.byref(mm), data, cap))
    return Message(mm.type, data.raw[:mm.data_len], mm.lower, mm.upper, mm.hash, mm.nonce)


def miner_handle(request_payload, devs=(0,)):
    """One GPU-miner step: Request payload -> Result payload (both Go JSON)."""
    p = _b(request_payload)
    arr = (ctypes.c_int * len(devs))(*devs)
    need = ctypes.c_size_t()
    buf = ctypes.create_string_buffer(256)
    _check(lib.mh_miner_handle(arr, len(devs), p, len(p), buf, 256, ctypes.byref(need)))
    return buf.raw[:need.value]


# ---- bitcoin/server/server.go (stub :62) mirror: include/minehip_server.h ----
from ._lib import mh_sched_opts, mh_assignment, mh_completion, mh_sched_stats  # noqa: E402


def _opts(init_chunk=None, min_chunk=None, max_chunk=None, target_ns=None):
    o = mh_sched_opts()
    lib.mh_sched_default_opts(ctypes.byref(o))
    for k, v in (("init_chunk", init_chunk), ("min_chunk", min_chunk), ("max_chunk", max_chunk),
                 ("target_ns", target_ns)):
        if v is not None:
            setattr(o, k, v)
    return o


def _stats(fn, h):
    st = mh_sched_stats()
    _check(fn(h, ctypes.byref(st)))
    return {f: int(getattr(st, f)) for f, _ in mh_sched_stats._fields_}


def _chk_neg(rc):
    if rc < 0:
        _check(rc)
    return rc


class Scheduler:
    """The server's chunk scheduler (mh_sched_*): jobs are client Requests,
    chunks go to miners, Results merge by the lexicographic min.  Times are
    caller-supplied nanoseconds."""

    def __init__(self, **opts):
        self._h = lib.mh_sched_create(ctypes.byref(_opts(**opts)))
        if not self._h:
            _check(MH_EINVAL)

    def close(self):
        if self._h:
            lib.mh_sched_destroy(self._h)
            self._h = None

    __del__ = close

    def add_miner(self, miner):
        _check(lib.mh_sched_add_miner(self._h, miner))

    def remove_miner(self, miner):
        _check(lib.mh_sched_remove_miner(self._h, miner))

    def submit(self, client, msg, lower, upper):
        m = _b(msg)
        return _chk_neg(lib.mh_sched_submit(self._h, client, m, len(m), lower, upper))

    def drop_client(self, client):
        return _chk_neg(lib.mh_sched_drop_client(self._h, client))

    def next(self, miner=-1, now=0):
        """(miner, job, lower, upper) or None."""
        a = mh_assignment()
        if _chk_neg(lib.mh_sched_next(self._h, miner, now, ctypes.byref(a))) == 0:
            return None
        return a.miner, a.job, a.lower, a.upper

    def job_msg(self, job):
        n = ctypes.c_size_t()
        buf = ctypes.create_string_buffer(MAX_MSG)
        _check(lib.mh_sched_job_msg(self._h, job, buf, MAX_MSG, ctypes.byref(n)))
        return buf.raw[:n.value]

    def result(self, miner, hash_, nonce, now=0):
        """(job, client, hash, nonce) when this Result finished its job, else None."""
        c = mh_completion()
        if _chk_neg(lib.mh_sched_result(self._h, miner, hash_, nonce, now, ctypes.byref(c))) == 0:
            return None
        return c.job, c.client, c.hash, c.nonce

    def stats(self):
        return _stats(lib.mh_sched_stats_read, self._h)


MAX_MSG = 1 << 20  # MH_MAX_MSG_LEN


class Server:
    """The server's message loop (mh_server_*): feed it what lsp.Server.Read
    returns, send what writes() yields with lsp.Server.Write."""

    def __init__(self, **opts):
        self._h = lib.mh_server_create(ctypes.byref(_opts(**opts)))
        if not self._h:
            _check(MH_EINVAL)
        self._buf = ctypes.create_string_buffer(4096)  # grown on demand (writes())

    def close(self):
        if self._h:
            lib.mh_server_destroy(self._h)
            self._h = None

    __del__ = close

    def read(self, conn, payload, now=0):
        p = _b(payload)
        _check(lib.mh_server_read(self._h, conn, p, len(p), now))

    def lost(self, conn, now=0):
        _check(lib.mh_server_lost(self._h, conn, now))

    def writes(self):
        """Drain the queued writes: list of (conn, payload bytes)."""
        out = []
        conn = ctypes.c_int64()
        n = ctypes.c_size_t()
        while True:
            rc = lib.mh_server_pop_write(self._h, ctypes.byref(conn), self._buf, len(self._buf), ctypes.byref(n))
            if rc == MH_EINVAL and n.value > len(self._buf):
                # an encoded Request can be ~6x its Data (JSON escapes): grow to the reported size
                self._buf = ctypes.create_string_buffer(n.value)
                continue
            if _chk_neg(rc) != 1:
                return out
            out.append((conn.value, self._buf.raw[:n.value]))

    def stats(self):
        return _stats(lib.mh_server_stats, self._h)
