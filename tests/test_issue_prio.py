"""CPU tests of the issue-priority build of fast_search:
the pass itself (csrc/issue_prio.py) and the code object embedded in
libminehip.so.  No GPU compute is called here."""
import ctypes
import os
import re
import shutil
import subprocess
import sys

import pytest

from conftest import PKG
from minehip import _lib

sys.path.insert(0, os.path.join(PKG, "csrc"))
import issue_prio  # noqa: E402

ASM = """\
\t.text
_ZN2mh11fast_searchILi4ELi0EEEvNS_8FastArgsEPNS_7PartialE:
\ts_load_dwordx4 s[0:3], s[4:5], 0x0
\tv_alignbit_b32 v1, v2, v2, 6
\tv_alignbit_b32 v3, v2, v2, 11
\tv_bitop3_b32 v4, v1, v3, v5 bitop3:0x96
\tv_add_u32_e32 v6, v4, v6
\ts_cmp_eq_u32 s0, 0
\tv_add3_u32 v7, v6, v4, v8
.LBB0_1:
\tv_add3_u32 v7, v6, v4, v8
\tv_xor_b32_e32 v9, v7, v9
\ts_endpgm
.Lfunc_end0:
\tv_alignbit_b32 v1, v2, v2, 6
"""


def test_markers_at_every_class_change():
    out, n = issue_prio.annotate(ASM)
    lines = out.split("\n")
    body = [ln.strip() for ln in lines]
    # half-rate run -> prio 3, full-rate run -> prio 0, again at the label (a branch may enter there)
    assert [b for b in body if b.startswith("s_setprio")] == \
        ["s_setprio 3", "s_setprio 0", "s_setprio 3", "s_setprio 3", "s_setprio 0"]
    assert n == 5
    i = body.index("v_alignbit_b32 v1, v2, v2, 6")
    assert body[i - 1] == "s_setprio 3"
    assert body[body.index("v_bitop3_b32 v4, v1, v3, v5 bitop3:0x96") - 1] == "s_setprio 0"
    # a full-rate op after a full-rate op: no marker between them
    assert body[body.index("v_add_u32_e32 v6, v4, v6") - 1].startswith("v_bitop3")


def test_only_markers_added():
    out, _ = issue_prio.annotate(ASM)
    assert [ln for ln in out.split("\n") if not ln.strip().startswith("s_setprio")] == ASM.split("\n")


def test_outside_kernels_untouched():
    out, _ = issue_prio.annotate(ASM)
    tail = out.split(".Lfunc_end0:")[1]
    assert "s_setprio" not in tail


def test_classes():
    # measured on MI355X (profiles/r01d_valu_ops.json, r03b_valu_ops.json)
    for op, c in (("v_alignbit_b32", "H"), ("v_add3_u32", "H"), ("v_lshrrev_b32_e64", "F"),
                  ("v_add_u32_e32", "F"), ("v_bitop3_b32", "F"), ("v_lshrrev_b32_e32", "F"),
                  ("v_lshlrev_b32_e32", "H"), ("v_cndmask_b32_e64", "H"), ("v_cndmask_b32_e32", "H"),
                  ("v_and_b32_e32", "F"), ("v_min_u32_dpp", "H"), ("v_cmp_lt_u32_e32", "H")):
        assert issue_prio.valu_class(f"\t{op} v1, v2, v3") == c, op
    assert issue_prio.valu_class("\ts_add_u32 s0, s1, s2") is None


def test_unknown_opcode_is_an_error():
    # an opcode in neither table must not default to a class
    with pytest.raises(issue_prio.UnknownOpcode):
        issue_prio.valu_class("\tv_lshl_add_u32_e64 v1, v2, 3, v4")
    with pytest.raises(issue_prio.UnknownOpcode):
        issue_prio.annotate(ASM.replace("v_xor_b32_e32 v9, v7, v9", "v_new_op_b32 v9, v7, v9"))


def test_unknown_opcode_fails_the_build_step(tmp_path):
    src = tmp_path / "in.s"
    src.write_text(ASM.replace("v_add_u32_e32 v6, v4, v6", "v_add_u32_sdwa v6, v4, v6"))
    r = subprocess.run([sys.executable, os.path.join(PKG, "csrc", "issue_prio.py"), str(src),
                        str(tmp_path / "out.s")], capture_output=True, text=True)
    assert r.returncode != 0
    assert "v_add_u32_sdwa" in r.stderr
    assert not (tmp_path / "out.s").exists()


def test_tables_are_disjoint_and_cover_the_real_build():
    from valu_rates import FULL, HALF
    assert not FULL & HALF
    asm = os.path.join(os.path.dirname(PKG), "build", "fast_search.s")
    if not os.path.exists(asm):
        pytest.skip("build/fast_search.s not built (make all)")
    ops = set(re.findall(r"^\s+(v_\w+)", open(asm).read(), flags=re.M))
    assert ops and ops <= FULL | HALF, sorted(ops - (FULL | HALF))
    # and the pass accepts the real compiler output as is
    _, n = issue_prio.annotate(open(asm).read())
    assert n > 10000


def embedded_code_object():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    begin = ctypes.addressof(ctypes.c_char.in_dll(lib, "mh_fast_co_begin"))
    end = ctypes.addressof(ctypes.c_char.in_dll(lib, "mh_fast_co_end"))
    assert end > begin
    return ctypes.string_at(begin, end - begin)


def test_embedded_code_object_is_a_gfx950_elf_with_every_variant():
    co = embedded_code_object()
    assert co[:4] == b"\x7fELF"
    assert int.from_bytes(co[18:20], "little") == 224  # EM_AMDGPU
    names = set(re.findall(rb"_ZN2mh11fast_searchILi(\d+)ELi(\d)EEEvNS_8FastArgsEPNS_7PartialE", co))
    want = {(str(j).encode(), b"0") for j in range(14)} | {(str(j).encode(), b"1") for j in range(5)} | \
        {(str(j).encode(), b"2") for j in (13, 14, 15)}
    assert want <= names


def test_embedded_code_object_carries_the_priority_markers(tmp_path):
    objdump = shutil.which("llvm-objdump") or "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not os.path.exists(objdump):
        pytest.skip("llvm-objdump not available")
    p = tmp_path / "fast.hsaco"
    p.write_bytes(embedded_code_object())
    dis = subprocess.run([objdump, "-d", "--mcpu=gfx950", str(p)], capture_output=True, text=True,
                         check=True).stdout
    prio = dis.count("s_setprio")
    valu = len(re.findall(r"^\s+v_\w+", dis, flags=re.M))
    # one marker per half-/full-rate run: hundreds per kernel (499 in fast_search<4,0>'s loop)
    assert prio > 10000 and prio < valu
