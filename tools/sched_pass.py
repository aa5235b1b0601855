"""Experimental post-RA reordering of the fast_search loop for the issue-priority
build: group half-rate and full-rate VALU instructions into
longer runs, so that a wave holds one priority for longer and fewer s_setprio
markers are needed.  Used through tools/isa_variant.py (variants sched_<D>_<R>).

Only "simple" VALU instructions move (one VGPR destination, register/constant
sources, no carry or lane ops); every other line is a barrier that nothing
crosses.  Within a segment the order respects every register dependency
(read-after-write, write-after-read, write-after-write).

  D  preferred distance (in instructions) between a producer and its consumer
  R  longest run of one class before switching when the other class is ready
"""
import re

MOVABLE = {
    "v_alignbit_b32", "v_bitop3_b32", "v_add3_u32", "v_add_u32_e32", "v_add_u32_e64", "v_lshrrev_b32_e32",
    "v_lshlrev_b32_e32", "v_xad_u32", "v_xor_b32_e32", "v_and_b32_e32", "v_or_b32_e32", "v_mov_b32_e32",
    "v_bfi_b32", "v_sub_u32_e32", "v_not_b32_e32",
}
HALF = {"v_alignbit_b32", "v_add3_u32", "v_xad_u32", "v_bfi_b32"}
TOK = re.compile(r"^(v|s)(\d+)$")


def parse(line):
    """(mnemonic, def register, use registers) of a movable instruction, else None."""
    m = re.match(r"^\s+(v_\w+)\s+(.*?)\s*(?:;.*)?$", line)
    if not m or m.group(1) not in MOVABLE:
        return None
    ops = [o.strip() for o in re.sub(r"\s+bitop3:0x[0-9a-fA-F]+$", "", m.group(2)).split(",")]
    regs = []
    for o in ops:
        t = TOK.match(o)
        if t:
            regs.append(o)
        elif re.match(r"^-?(\d+|0x[0-9a-fA-F]+)$", o):
            continue
        else:
            return None  # anything else (ranges, vcc, modifiers): do not move it
    if not regs or not regs[0].startswith("v"):
        return None
    return m.group(1), regs[0], set(regs[1:])


def schedule_segment(items, D, R, raw_only=False):
    """items: list of (line, mnemonic, def, uses).  Returns the reordered lines.  raw_only drops the
    write-after-read / write-after-write edges: the result is WRONG (registers are reused), only
    its timing means something -- an upper bound for grouping with register renaming."""
    n = len(items)
    preds = [set() for _ in range(n)]
    last_def, last_uses = {}, {}
    for i, (_, _, d, uses) in enumerate(items):
        for u in uses:
            if u in last_def:
                preds[i].add(last_def[u])          # RAW
        if d in last_def and not raw_only:
            preds[i].add(last_def[d])              # WAW
        for j in (() if raw_only else last_uses.get(d, ())):
            if j != i:
                preds[i].add(j)                    # WAR
        for u in uses:
            last_uses.setdefault(u, set()).add(i)
        last_def[d] = i
        last_uses[d] = set()
    succs = [[] for _ in range(n)]
    for i in range(n):
        for p in preds[i]:
            succs[p].append(i)
    prio = [0] * n
    for i in reversed(range(n)):
        prio[i] = 1 + max((prio[s] for s in succs[i]), default=0)
    cls = ["H" if it[1] in HALF else "F" for it in items]
    npred = [len(p) for p in preds]
    ready_at = [0] * n
    avail = {i for i in range(n) if npred[i] == 0}
    out, cur, run = [], None, 0
    pos = 0
    while avail:
        now = [i for i in avail if ready_at[i] <= pos]
        pool = now or [min(avail, key=lambda i: (ready_at[i], -prio[i], i))]
        same = [i for i in pool if cls[i] == cur]
        if same and run < R:
            pick = max(same, key=lambda i: (prio[i], -i))
        else:
            other = [i for i in pool if cls[i] != cur]
            pick = max(other or pool, key=lambda i: (prio[i], -i))
        avail.remove(pick)
        out.append(pick)
        run = run + 1 if cls[pick] == cur else 1
        cur = cls[pick]
        for s in succs[pick]:
            npred[s] -= 1
            ready_at[s] = max(ready_at[s], pos + D)
            if npred[s] == 0:
                avail.add(s)
        pos += 1
    assert len(out) == n
    return [items[i][0] for i in out]


def reorder(text, D=2, R=8, min_block=200, raw_only=False):
    """Reorder the large basic blocks of the fast_search kernels.  Returns (text, moved blocks)."""
    lines = text.split("\n")
    out, block, nblk = [], [], 0

    def flush():
        nonlocal nblk
        nv = sum(1 for ln in block if re.match(r"^\s+v_", ln))
        if nv < min_block:
            out.extend(block)
            return
        nblk += 1
        seg = []
        for ln in block:
            p = parse(ln)
            if p is None:
                if seg:
                    out.extend(schedule_segment(seg, D, R, raw_only))
                    seg = []
                out.append(ln)
            else:
                seg.append((ln,) + p)
        if seg:
            out.extend(schedule_segment(seg, D, R, raw_only))

    in_kernel = False
    for ln in lines:
        starts = re.match(r"^_Z\S+:", ln) or re.match(r"^\.LBB\w*:", ln) or ln.startswith(".Lfunc_end")
        if starts:
            flush()
            block = []
            if re.match(r"^_Z\S+:", ln):
                in_kernel = "fast_search" in ln
            elif ln.startswith(".Lfunc_end"):
                in_kernel = False
        if in_kernel:
            block.append(ln)
        else:
            out.append(ln)
    flush()
    return "\n".join(out), nblk
