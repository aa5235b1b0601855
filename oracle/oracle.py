"""ctypes binding of the CPU restatement (oracle/sha256_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product path (minehip package,
libminehip.so).  See sha256_oracle.c for the reference file:line each function
restates.
"""
import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "liboracle_sha256.so")
_SO_OSSL = os.path.join(_HERE, "liboracle_openssl.so")
_lib = None
_lib_ossl = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        u8p = ctypes.c_char_p
        u64 = ctypes.c_uint64
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.oracle_sha256.argtypes = [u8p, ctypes.c_size_t, ctypes.c_char_p]
        L.oracle_hash.argtypes = [u8p, ctypes.c_size_t, u64]
        L.oracle_hash.restype = u64
        L.oracle_hash_batch.argtypes = [u8p, ctypes.c_size_t, u64p, ctypes.c_size_t, u64p]
        L.oracle_search.argtypes = [u8p, ctypes.c_size_t, u64, u64, u64p, u64p]
        L.oracle_search.restype = ctypes.c_int
        L.oracle_search_mt.argtypes = [u8p, ctypes.c_size_t, u64, u64, ctypes.c_int, u64p, u64p]
        L.oracle_search_mt.restype = ctypes.c_int
        _lib = L
    return _lib


def _b(msg):
    return msg.encode("utf-8") if isinstance(msg, str) else bytes(msg)


def sha256(data):
    data = _b(data)
    out = ctypes.create_string_buffer(32)
    lib().oracle_sha256(data, len(data), out)
    return out.raw


def hash_(msg, nonce):
    """bitcoin/hash.go:13-17"""
    m = _b(msg)
    return lib().oracle_hash(m, len(m), nonce)


def hash_batch(msg, nonces):
    import numpy as np
    m = _b(msg)
    a = np.ascontiguousarray(nonces, dtype=np.uint64)
    out = np.empty_like(a)
    p = ctypes.POINTER(ctypes.c_uint64)
    lib().oracle_hash_batch(m, len(m), a.ctypes.data_as(p), a.size, out.ctypes.data_as(p))
    return out


def search(msg, lower, upper, threads=1):
    """Scan spec of SURVEY.md §8(a) A2 (reference stub miner.go:33)."""
    m = _b(msg)
    h = ctypes.c_uint64()
    n = ctypes.c_uint64()
    if threads <= 1:
        rc = lib().oracle_search(m, len(m), lower, upper, ctypes.byref(h), ctypes.byref(n))
    else:
        rc = lib().oracle_search_mt(m, len(m), lower, upper, threads, ctypes.byref(h), ctypes.byref(n))
    if rc != 0:
        raise ValueError("oracle_search: lower > upper")
    return h.value, n.value


def search_openssl(msg, lower, upper, threads=1):
    """Optimised CPU scan (openssl_scan.c: midstate + OpenSSL SHA-256), same
    answer as search(); bench.py's tuned CPU baseline."""
    global _lib_ossl
    if _lib_ossl is None:
        if not os.path.exists(_SO_OSSL):
            build()
        L = ctypes.CDLL(_SO_OSSL)
        u64 = ctypes.c_uint64
        L.oracle_search_openssl.argtypes = [ctypes.c_char_p, ctypes.c_size_t, u64, u64, ctypes.c_int,
                                            ctypes.POINTER(u64), ctypes.POINTER(u64)]
        L.oracle_search_openssl.restype = ctypes.c_int
        _lib_ossl = L
    m = _b(msg)
    h = ctypes.c_uint64()
    n = ctypes.c_uint64()
    if _lib_ossl.oracle_search_openssl(m, len(m), lower, upper, threads, ctypes.byref(h), ctypes.byref(n)) != 0:
        raise ValueError("oracle_search_openssl: lower > upper")
    return h.value, n.value
