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

import msgpack

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
                return msgpack.unpackb(co[d:d + descsz], raw=False, strict_map_key=False)
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
