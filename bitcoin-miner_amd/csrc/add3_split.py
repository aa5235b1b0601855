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


def _reads(line, reg):
    """Whether an instruction line reads register `reg` (any operand after the destination)."""
    m = re.match(r"^\s+([sv]_\w+)\s+(.*)$", line)
    if not m:
        return False
    ops = [o.strip() for o in m.group(2).split(",")]
    return any(re.fullmatch(reg, o) for o in ops[1:])


def split_by_slack(text, frac, horizon=400):
    """Split the fraction `frac` of each fast kernel's add3s whose results are read latest: the
    distance, in VALU instructions, from the add3 to the first instruction reading its destination
    (two dependent adds take one more issue slot on that chain than one add3).  Returns (text, n)."""
    lines = text.split("\n")
    out, n = [], 0
    i = 0
    while i < len(lines):
        if not re.match(r"^_ZN2mh11fast_search\S*:", lines[i]):
            out.append(lines[i])
            i += 1
            continue
        j = i
        while j < len(lines) and not lines[j].startswith(".Lfunc_end"):
            j += 1
        body = lines[i:j]
        cand = []
        for a, ln in enumerate(body):
            m = ADD3.match(ln)
            if not m:
                continue
            d, dist = m.group(2), horizon
            seen = 0
            for b in range(a + 1, min(len(body), a + 1 + 4 * horizon)):
                if body[b].strip().startswith("v_"):
                    seen += 1
                if _reads(body[b], re.escape(d)) or seen >= horizon:
                    dist = seen
                    break
            cand.append((dist, a))
        k = int(round(frac * len(cand)))
        pick = {a for _, a in sorted(cand, key=lambda t: (-t[0], t[1]))[:k]}
        for a, ln in enumerate(body):
            rep = split_line(ADD3.match(ln)) if a in pick else None
            if rep is not None:
                out.extend(rep)
                n += 1
            else:
                out.append(ln)
        i = j
    return "\n".join(out), n


def main():
    k, src, dst = int(sys.argv[1]), sys.argv[2], sys.argv[3]
    text, n = split(open(src).read(), k)
    open(dst, "w").write(text)
    print(f"add3_split: {n} v_add3_u32 of the fast kernels split (every {k}th of each) -> {dst}")


if __name__ == "__main__":
    main()
