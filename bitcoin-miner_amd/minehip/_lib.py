"""ctypes binding of libminehip.so (C-ABI: include/minehip.h, include/minehip_server.h).

The library is built in-tree (``make`` at the repo root, or
``__graft_entry__.build()``) next to this file.  There is no fallback: if the
shared object is missing, importing this module raises.

MINEHIP_LIB names another build of the same ABI to load instead -- the dev
build (``make dev``: build/dev/libminehip.so, with the experiment and test
hooks) for tools/kbench.py A/Bs and the GPU tests that inject failures.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
PRODUCT_LIB_PATH = os.path.join(_HERE, "libminehip.so")
LIB_PATH = os.environ.get("MINEHIP_LIB") or PRODUCT_LIB_PATH

MH_OK = 0
MH_EINVAL = -1
MH_ERANGE = -2
MH_ETOOLONG = -3
MH_ENODEV = -4
MH_EHIP = -5
MH_ENOTREQ = -6
MH_EINTERNAL = -7
MH_EREJECTED = -8
OPS_PER_BLOCK = 1376  # MH_OPS_PER_BLOCK
MH_ABI_VERSION = 5    # include/minehip.h: the struct layouts below are this version's
MH_MAX_WORKERS = 256  # most devices one mh_search_multi / mh_multi_plan call may list

#: every symbol include/*.h declares
EXPORTS = (
    "mh_abi_version", "mh_device_count", "mh_search", "mh_search_multi", "mh_hash_batch",
    "mh_last_error", "mh_msg_encode", "mh_msg_decode", "mh_miner_handle",
    "mh_profile_enable", "mh_profile_read", "mh_profile_kernels", "mh_plan", "mh_multi_plan",
    "mh_multi_rates",
    # minehip_server.h
    "mh_sched_default_opts", "mh_sched_create", "mh_sched_destroy", "mh_sched_add_miner",
    "mh_sched_remove_miner", "mh_sched_submit", "mh_sched_drop_client", "mh_sched_next",
    "mh_sched_job_msg", "mh_sched_result", "mh_sched_stats_read",
    "mh_server_create", "mh_server_destroy", "mh_server_read", "mh_server_lost",
    "mh_server_pop_write", "mh_server_stats",
)


class mh_piece(ctypes.Structure):
    _fields_ = [("first", ctypes.c_uint64), ("count", ctypes.c_uint64), ("kind", ctypes.c_int32),
                ("digits", ctypes.c_int32), ("lo_digits", ctypes.c_int32), ("word", ctypes.c_int32),
                ("mode", ctypes.c_int32), ("blocks", ctypes.c_int32), ("nonce_ops", ctypes.c_uint32),
                ("nonce_slots", ctypes.c_uint32)]


class mh_kernel_stat(ctypes.Structure):
    _fields_ = [("word", ctypes.c_int32), ("mode", ctypes.c_int32), ("launches", ctypes.c_uint64),
                ("nonces", ctypes.c_uint64), ("ns", ctypes.c_uint64), ("ops", ctypes.c_uint64),
                ("slots", ctypes.c_uint64), ("lo_digits", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class mh_span(ctypes.Structure):
    _fields_ = [("lower", ctypes.c_uint64), ("upper", ctypes.c_uint64), ("worker", ctypes.c_int32),
                ("kind", ctypes.c_int32), ("cost", ctypes.c_double)]


class mh_message(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int64), ("lower", ctypes.c_uint64), ("upper", ctypes.c_uint64),
                ("hash", ctypes.c_uint64), ("nonce", ctypes.c_uint64), ("data_len", ctypes.c_size_t)]


class mh_sched_opts(ctypes.Structure):
    _fields_ = [("init_chunk", ctypes.c_uint64), ("min_chunk", ctypes.c_uint64),
                ("max_chunk", ctypes.c_uint64), ("target_ns", ctypes.c_uint64)]


class mh_assignment(ctypes.Structure):
    _fields_ = [("miner", ctypes.c_int64), ("job", ctypes.c_int64), ("lower", ctypes.c_uint64),
                ("upper", ctypes.c_uint64), ("msg_len", ctypes.c_size_t)]


class mh_completion(ctypes.Structure):
    _fields_ = [("job", ctypes.c_int64), ("client", ctypes.c_int64), ("hash", ctypes.c_uint64),
                ("nonce", ctypes.c_uint64)]


class mh_sched_stats(ctypes.Structure):
    _fields_ = [(f, ctypes.c_uint64) for f in (
        "miners", "idle_miners", "jobs", "chunks_assigned", "chunks_done", "chunks_requeued",
        "nonces_done", "jobs_done", "jobs_cancelled")]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libminehip.so not found at {LIB_PATH}; build it with `make` at the repo root "
            "(hipcc --offload-arch=gfx950).  There is no CPU fallback.")
    L = ctypes.CDLL(LIB_PATH)
    L.mh_abi_version.restype = ctypes.c_int
    got = L.mh_abi_version()
    if got != MH_ABI_VERSION:
        # a library of another ABI would read and write these structs at other strides
        raise ImportError(f"{LIB_PATH} has ABI {got}, this binding needs {MH_ABI_VERSION}: rebuild (make)")
    u8p = ctypes.c_char_p
    sz = ctypes.c_size_t
    u64 = ctypes.c_uint64
    u64p = ctypes.POINTER(ctypes.c_uint64)
    intp = ctypes.POINTER(ctypes.c_int)
    L.mh_abi_version.restype = ctypes.c_int
    L.mh_device_count.restype = ctypes.c_int
    L.mh_last_error.restype = ctypes.c_char_p
    L.mh_search.argtypes = [ctypes.c_int, u8p, sz, u64, u64, u64p, u64p]
    L.mh_search_multi.argtypes = [intp, ctypes.c_int, u8p, sz, u64, u64, u64, u64p, u64p]
    L.mh_hash_batch.argtypes = [ctypes.c_int, u8p, sz, u64p, sz, u64p]
    L.mh_msg_encode.argtypes = [ctypes.c_int64, u8p, sz, u64, u64, u64, u64, ctypes.c_char_p, sz,
                                ctypes.POINTER(sz)]
    L.mh_msg_decode.argtypes = [ctypes.c_char_p, sz, ctypes.POINTER(mh_message), ctypes.c_char_p, sz]
    L.mh_miner_handle.argtypes = [intp, ctypes.c_int, ctypes.c_char_p, sz, ctypes.c_char_p, sz,
                                  ctypes.POINTER(sz)]
    L.mh_profile_enable.argtypes = [ctypes.c_int, ctypes.c_int]
    L.mh_profile_read.argtypes = [ctypes.c_int, u64p, ctypes.c_int]
    L.mh_profile_kernels.argtypes = [ctypes.c_int, ctypes.POINTER(mh_kernel_stat), ctypes.c_int]
    L.mh_plan.argtypes = [u8p, sz, u64, u64, ctypes.POINTER(mh_piece), ctypes.c_int64]
    L.mh_plan.restype = ctypes.c_int64
    L.mh_multi_plan.argtypes = [u8p, sz, u64, u64, ctypes.POINTER(ctypes.c_double), ctypes.c_int,
                                ctypes.POINTER(mh_span), ctypes.c_int64]
    L.mh_multi_rates.argtypes = [intp, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    vp = ctypes.c_void_p
    i64 = ctypes.c_int64
    L.mh_sched_default_opts.argtypes = [ctypes.POINTER(mh_sched_opts)]
    L.mh_sched_create.argtypes = [ctypes.POINTER(mh_sched_opts)]
    L.mh_sched_destroy.argtypes = [vp]
    L.mh_sched_add_miner.argtypes = [vp, i64]
    L.mh_sched_remove_miner.argtypes = [vp, i64]
    L.mh_sched_submit.argtypes = [vp, i64, u8p, sz, u64, u64]
    L.mh_sched_drop_client.argtypes = [vp, i64]
    L.mh_sched_next.argtypes = [vp, i64, u64, ctypes.POINTER(mh_assignment)]
    L.mh_sched_job_msg.argtypes = [vp, i64, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
    L.mh_sched_result.argtypes = [vp, i64, u64, u64, u64, ctypes.POINTER(mh_completion)]
    L.mh_sched_stats_read.argtypes = [vp, ctypes.POINTER(mh_sched_stats)]
    L.mh_server_create.argtypes = [ctypes.POINTER(mh_sched_opts)]
    L.mh_server_destroy.argtypes = [vp]
    L.mh_server_read.argtypes = [vp, i64, ctypes.c_char_p, sz, u64]
    L.mh_server_lost.argtypes = [vp, i64, u64]
    L.mh_server_pop_write.argtypes = [vp, ctypes.POINTER(i64), ctypes.c_char_p, sz, ctypes.POINTER(sz)]
    L.mh_server_stats.argtypes = [vp, ctypes.POINTER(mh_sched_stats)]
    restype = {"mh_plan": ctypes.c_int64, "mh_multi_plan": ctypes.c_int64, "mh_last_error": ctypes.c_char_p, "mh_sched_submit": i64,
               "mh_sched_create": vp, "mh_server_create": vp, "mh_sched_default_opts": None,
               "mh_sched_destroy": None, "mh_server_destroy": None}
    for name in EXPORTS:
        getattr(L, name).restype = restype.get(name, ctypes.c_int)
    return L


lib = _load()
