"""issue_prio.py -- the issue-priority pass of the fast_search build (Makefile).

    python3 issue_prio.py in.s out.s

Reads the gfx950 assembly of fast_search.hip and, inside every kernel, puts
`s_setprio 3` before each run of half-rate VALU instructions and
`s_setprio 0` before each run of full-rate ones.  Nothing else changes: no
instruction is moved, added or removed besides the s_setprio markers.

Why (profiles/r02p..r): a gfx950 SIMD issues one VALU
instruction per quad-cycle, or two when both are full rate -- and a
full-rate op can also go beside a half-rate op from another wave.  Under
age-ordered arbitration the waves that are not the oldest sit at half-rate
heads, so the loop's full-rate ops (41%) almost never find a partner (5.3% of
quad-cycles issued two).  With the markers, a wave about to issue full-rate ops
drops below the waves that are in a half-rate run, and its full-rate ops then
issue beside their half-rate ones: the SHA-256 round mix goes from 4.07 to
3.20 cycles per instruction, the kernel from 33.9 to 50.0 GH/s.

s_setprio is a scalar instruction (it changes the wave's own arbitration
priority only; no memory, no data).
"""
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from valu_rates import UnknownOpcode, valu_rate  # noqa: E402  (the opcode tables)

PRIO_HALF, PRIO_FULL = 3, 0


def valu_class(line):
    """'H' / 'F' for a VALU instruction line, None for any other line;
    UnknownOpcode for a VALU opcode valu_rates.py does not list."""
    m = re.match(r"^\s+(v_\w+)", line)
    if not m:
        return None
    return valu_rate(m.group(1))


def annotate(text):
    """Returns (annotated text, markers inserted)."""
    out, n, cur, in_kernel = [], 0, None, False
    for line in text.split("\n"):
        if re.match(r"^_Z\S+:", line):        # kernel entry
            in_kernel, cur = True, None
        elif line.startswith(".Lfunc_end"):
            in_kernel = False
        elif re.match(r"^\.LBB\w*:", line):    # block start: a branch may enter here
            cur = None
        if in_kernel:
            c = valu_class(line)
            if c is not None and c != cur:
                out.append(f"\ts_setprio {PRIO_HALF if c == 'H' else PRIO_FULL}")
                n += 1
                cur = c
        out.append(line)
    return "\n".join(out), n


def main():
    src, dst = sys.argv[1], sys.argv[2]
    try:
        text, n = annotate(open(src).read())
    except UnknownOpcode as e:
        sys.exit(f"issue_prio: {src}: {e}")
    if n == 0:
        sys.exit("issue_prio: no VALU instruction found in " + src)
    open(dst, "w").write(text)
    print(f"issue_prio: {n} s_setprio markers -> {dst}")


if __name__ == "__main__":
    main()
