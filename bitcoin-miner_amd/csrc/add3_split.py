"""add3_split.py -- the add3 split of the fast_search build (Makefile, before issue_prio.py).

    python3 add3_split.py K in.s out.s

Inside every fast_search kernel of the gfx950 assembly, every K-th `v_add3_u32 d, a, b, c`
(counted from the kernel's entry) becomes two full-rate adds, `d = x + y; d = z + d`, where z is
an operand other than d, so the first add cannot overwrite it.  Nothing else changes.

Why: a half-rate op never shares its quad-cycle with another half-rate op, so the
per-nonce loop needs at least max(H, N/2) quad-cycles (H half-rate of N instructions; 701 of
1,196 for fast_search<4, One>).  Trading an add3 (one H) for two adds (two F) lowers that bound at
the price of one more instruction.  The chip runs this kernel at its power limit, so fewer
quad-cycles per nonce come back partly as a lower clock; measured with the in-kernel clock probe,
every 4th add3 split ran 5% fewer quad-cycles per nonce at a 4% lower clock.
"""
import re
import sys

ADD3 = re.compile(r"^(\s+)v_add3_u32\s+(\S+),\s*(\S+),\s*(\S+),\s*(\S+)\s*$")


def is_vgpr(op):
    return re.match(r"^v\d+$", op) is not None


def split_line(m):
    """The two adds replacing one matched v_add3_u32, or None when every source is the
    destination (no operand may go last)."""
    ind, d, a, b, c = m.groups()
    ops = [a, b, c]
    last = next((x for x in reversed(ops) if x != d), None)
    if last is None:
        return None
    ops.remove(last)
    x, y = ops
    if is_vgpr(y):        # VOP2: src1 must be a VGPR, src0 may be anything
        first = f"{ind}v_add_u32_e32 {d}, {x}, {y}"
    elif is_vgpr(x):
        first = f"{ind}v_add_u32_e32 {d}, {y}, {x}"
    else:
        first = f"{ind}v_add_u32_e64 {d}, {x}, {y}"
    return [first, f"{ind}v_add_u32_e32 {d}, {last}, {d}"]


def split(text, k, pattern=None):
    """Returns (text, add3 split).  Splits every k-th v_add3 of each fast kernel (k <= 0: none),
    or, with `pattern` (a string of 0/1 repeated over each kernel's add3s, e.g. "001" = k 3),
    those at a '1'."""
    if pattern is None:
        if k <= 0:
            return text, 0
        pattern = "0" * (k - 1) + "1"
    if "1" not in pattern:
        return text, 0
    out, n, i, inside = [], 0, 0, False
    for line in text.split("\n"):
        if re.match(r"^_ZN2mh11fast_search\S*:", line):
            inside, i = True, 0
        elif line.startswith(".Lfunc_end"):
            inside = False
        m = ADD3.match(line) if inside else None
        if m:
            i += 1
            if pattern[(i - 1) % len(pattern)] == "1":
                rep = split_line(m)
                if rep is not None:
                    out.extend(rep)
                    n += 1
                    continue
        out.append(line)
    return "\n".join(out), n


def main():
    k, src, dst = int(sys.argv[1]), sys.argv[2], sys.argv[3]
    text, n = split(open(src).read(), k)
    open(dst, "w").write(text)
    print(f"add3_split: {n} v_add3_u32 of the fast kernels split (every {k}th of each) -> {dst}")


if __name__ == "__main__":
    main()
