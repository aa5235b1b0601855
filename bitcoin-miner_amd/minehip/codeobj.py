"""Register and memory resources of the fast_search kernels, read from the
code object embedded in libminehip.so (mh_fast_co_begin .. mh_fast_co_end,
csrc/fast_co.S) -- the very bytes each device loads with hipModuleLoadData.

The AMDGPU ELF carries an NT_AMDGPU_METADATA note (msgpack, code object v5)
with one map per kernel: .vgpr_count, .sgpr_count, .agpr_count,
.private_segment_fixed_size (scratch bytes per lane), .group_segment_fixed_size
(static LDS), spill counts.  Host-only: no GPU is touched.
"""
import ctypes
import struct

from ._lib import lib

NT_AMDGPU_METADATA = 32
SHT_NOTE = 7
VGPRS_PER_SIMD_LANE = 512     # gfx950: unified VGPR + AGPR file, per lane of a SIMD (wave64)
VGPR_GRANULE = 8              # allocation granule
MAX_WAVES_PER_SIMD = 8


def fast_code_object():
    """The embedded code object's bytes."""
    b = ctypes.addressof(ctypes.c_ubyte.in_dll(lib, "mh_fast_co_begin"))
    e = ctypes.addressof(ctypes.c_ubyte.in_dll(lib, "mh_fast_co_end"))
    return ctypes.string_at(b, e - b)


def unpack_msgpack(b):
    """Decode one MessagePack object (the subset AMDGPU metadata uses: maps, arrays, strings,
    binary, integers, floats, booleans, nil).  No dependency on the msgpack package."""
    def rd(i):
        t = b[i]
        if t <= 0x7F:
            return t, i + 1
        if t >= 0xE0:
            return t - 0x100, i + 1
        if 0x80 <= t <= 0x8F:
            return rd_map(i + 1, t & 0x0F)
        if 0x90 <= t <= 0x9F:
            return rd_arr(i + 1, t & 0x0F)
        if 0xA0 <= t <= 0xBF:
            n = t & 0x1F
            return b[i + 1:i + 1 + n].decode(), i + 1 + n
        if t == 0xC0:
            return None, i + 1
        if t in (0xC2, 0xC3):
            return t == 0xC3, i + 1
        if t in (0xC4, 0xC5, 0xC6, 0xD9, 0xDA, 0xDB):      # bin8/16/32, str8/16/32
            w = {0xC4: 1, 0xC5: 2, 0xC6: 4, 0xD9: 1, 0xDA: 2, 0xDB: 4}[t]
            n = int.from_bytes(b[i + 1:i + 1 + w], "big")
            v = b[i + 1 + w:i + 1 + w + n]
            return (v.decode() if t >= 0xD9 else bytes(v)), i + 1 + w + n
        if t in (0xCA, 0xCB):
            return struct.unpack(">f" if t == 0xCA else ">d", b[i + 1:i + (5 if t == 0xCA else 9)])[0], \
                i + (5 if t == 0xCA else 9)
        if 0xCC <= t <= 0xD3:                               # uint8..64, int8..64
            w = 1 << ((t - 0xCC) % 4)
            return int.from_bytes(b[i + 1:i + 1 + w], "big", signed=t >= 0xD0), i + 1 + w
        if t in (0xDC, 0xDD, 0xDE, 0xDF):                   # array16/32, map16/32
            w = 2 if t in (0xDC, 0xDE) else 4
            n = int.from_bytes(b[i + 1:i + 1 + w], "big")
            return (rd_arr if t < 0xDE else rd_map)(i + 1 + w, n)
        raise ValueError(f"msgpack type 0x{t:02x} not supported")

    def rd_arr(i, n):
        out = []
        for _ in range(n):
            v, i = rd(i)
            out.append(v)
        return out, i

    def rd_map(i, n):
        out = {}
        for _ in range(n):
            k, i = rd(i)
            v, i = rd(i)
            out[k] = v
        return out, i

    return rd(0)[0]


def metadata(co):
    """The decoded NT_AMDGPU_METADATA note of an AMDGPU ELF64 code object."""
    if co[:4] != b"\x7fELF" or co[4] != 2:
        raise ValueError("not an ELF64 code object")
    shoff = struct.unpack_from("<Q", co, 0x28)[0]
    shentsize, shnum = struct.unpack_from("<HH", co, 0x3A)
    for i in range(shnum):
        _, typ, _, _, off, size = struct.unpack_from("<IIQQQQ", co, shoff + i * shentsize)
        if typ != SHT_NOTE:
            continue
        p = off
        while p + 12 <= off + size:
            namesz, descsz, ntype = struct.unpack_from("<III", co, p)
            name = co[p + 12:p + 12 + namesz].rstrip(b"\0")
            d = p + 12 + ((namesz + 3) & ~3)
            if name == b"AMDGPU" and ntype == NT_AMDGPU_METADATA:
                return unpack_msgpack(co[d:d + descsz])
            p = d + ((descsz + 3) & ~3)
    raise ValueError("no NT_AMDGPU_METADATA note")


def max_waves_per_simd(vgpr, agpr=0):
    """Waves a SIMD can hold by register file alone (gfx950: 512 unified
    registers per lane, 8-register granules, at most 8 waves)."""
    alloc = -(-(vgpr + agpr) // VGPR_GRANULE) * VGPR_GRANULE
    return min(MAX_WAVES_PER_SIMD, VGPRS_PER_SIMD_LANE // max(alloc, VGPR_GRANULE))


def fast_kernel_resources():
    """{(J, MODE): {vgpr, sgpr, agpr, scratch_bytes, lds_bytes, spills, max_waves_per_simd}}."""
    import re
    out = {}
    for k in metadata(fast_code_object())["amdhsa.kernels"]:
        m = re.match(r"_ZN2mh11fast_searchILi(\d+)ELi(\d+)E", k[".name"])
        if not m:
            continue
        out[(int(m.group(1)), int(m.group(2)))] = {
            "vgpr": k[".vgpr_count"], "sgpr": k[".sgpr_count"], "agpr": k.get(".agpr_count", 0),
            "scratch_bytes": k[".private_segment_fixed_size"], "lds_bytes": k[".group_segment_fixed_size"],
            "vgpr_spills": k.get(".vgpr_spill_count", 0), "sgpr_spills": k.get(".sgpr_spill_count", 0),
            "max_waves_per_simd": max_waves_per_simd(k[".vgpr_count"], k.get(".agpr_count", 0)),
        }
    return out
