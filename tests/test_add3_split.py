"""CPU tests of the add3 split of the fast_search build (csrc/add3_split.py): every
K-th v_add3_u32 of a fast kernel becomes two full-rate adds computing the same value, whatever
its operands alias; nothing outside the fast kernels changes."""
import os
import random
import re
import sys

import pytest

from conftest import PKG

sys.path.insert(0, os.path.join(PKG, "csrc"))
import add3_split  # noqa: E402

M32 = (1 << 32) - 1


def run(lines, regs):
    """Execute v_add3_u32 / v_add_u32_e32 / v_add_u32_e64 lines on a register dict."""
    regs = dict(regs)

    def val(op):
        return regs[op] if op in regs else int(op, 0) & M32

    for ln in lines:
        m = re.match(r"^\s+(v_add3_u32|v_add_u32_e32|v_add_u32_e64)\s+(.*)$", ln)
        assert m, ln
        d, *src = [x.strip() for x in m.group(2).split(",")]
        if m.group(1) == "v_add_u32_e32":
            assert re.match(r"^v\d+$", src[1]), ln   # VOP2: src1 is a VGPR
        regs[d] = sum(val(s) for s in src) & M32
    return regs


OPERANDS = ["v1", "v2", "v3", "s4", "7", "-3"]


@pytest.mark.parametrize("seed", range(3))
def test_split_computes_the_same_sum_under_any_aliasing(seed):
    rng = random.Random(seed)
    for _ in range(300):
        d = rng.choice(["v1", "v2", "v3"])
        a, b, c = (rng.choice(OPERANDS) for _ in range(3))
        line = f"\tv_add3_u32 {d}, {a}, {b}, {c}"
        regs = {r: rng.randrange(1 << 32) for r in ("v1", "v2", "v3", "s4")}
        rep = add3_split.split_line(add3_split.ADD3.match(line))
        if rep is None:                               # every source is the destination
            assert a == b == c == d
            continue
        assert len(rep) == 2 and all("v_add3" not in r for r in rep)
        assert run(rep, regs) == run([line], regs), (line, rep)


ASM = """\
\t.text
_ZN2mh11fast_searchILi4ELi0EEEvNS_8FastArgsEPNS_7PartialE:
\tv_add3_u32 v1, v2, v3, v4
\tv_add3_u32 v5, v1, v3, v4
\tv_add3_u32 v6, v5, s2, v6
\tv_add3_u32 v7, v6, v1, v1
.Lfunc_end0:
_ZN2mh12generic_scanEv:
\tv_add3_u32 v1, v2, v3, v4
\tv_add3_u32 v1, v2, v3, v4
.Lfunc_end1:
_ZN2mh11fast_searchILi3ELi0EEEvNS_8FastArgsEPNS_7PartialE:
\tv_add3_u32 v1, v2, v3, v4
\tv_add3_u32 v5, v1, v3, v4
.Lfunc_end2:
"""


def test_every_kth_add3_of_each_fast_kernel_only():
    out, n = add3_split.split(ASM, 2)
    assert n == 3                                     # 2 in the first fast kernel, 1 in the second
    kernels = out.split(".Lfunc_end")
    assert kernels[0].count("v_add3_u32") == 2 and kernels[0].count("v_add_u32") == 4
    assert kernels[1].count("v_add3_u32") == 2         # generic_scan untouched
    assert kernels[2].count("v_add3_u32") == 1         # the count restarts at each kernel
    assert add3_split.split(ASM, 0) == (ASM, 0)


def test_build_uses_the_split():
    """The Makefile runs the pass between the compiler's assembly and the issue-priority pass."""
    mk = open(os.path.join(os.path.dirname(PKG), "Makefile")).read()
    assert "add3_split.py" in mk


def test_split_by_slack_picks_the_results_read_latest():
    body = ["\tv_add3_u32 v1, v2, v3, v4",      # read by the very next instruction
            "\tv_xor_b32_e32 v9, v1, v9",
            "\tv_add3_u32 v5, v2, v3, v4"]     # read only after ten more instructions
    body += [f"\tv_xor_b32_e32 v{10 + i}, v2, v3" for i in range(10)]
    body += ["\tv_add_u32_e32 v6, v5, v6"]
    asm = "_ZN2mh11fast_searchILi4ELi0EEEvNS_8FastArgsEPNS_7PartialE:\n" + "\n".join(body) + "\n.Lfunc_end0:\n"
    out, n = add3_split.split_by_slack(asm, 0.5)
    assert n == 1
    assert "v_add3_u32 v1, v2, v3, v4" in out and "v_add3_u32 v5" not in out
    assert add3_split.split_by_slack(asm, 0.0) == (asm, 0)
