"""Per-kernel register use and per-nonce issue cost from the gfx950 assembly.

  make asm && python tools/isa_report.py build/fast_search_prio.s [filter]

For every kernel: VGPRs/SGPRs/scratch from the metadata, and for the
largest loop body (the per-nonce body of fast_search) the VALU instruction count,
split into full-rate and half-rate instructions as measured by tools/valu_ops.hip
on MI355X, the issue-priority markers in the loop, and the mix bound: the share
of the 2-per-quad-cycle issue peak the loop's mix can reach (a half-rate op
cannot share its quad-cycle with another half-rate op).
"""
import re
import sys
from collections import Counter

import os  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "bitcoin-miner_amd", "csrc"))
from valu_rates import HALF as HALF_RATE  # noqa: E402  (one table with the issue-priority pass)
from loop_mix import inner_loop, kernels  # noqa: E402  (the loop finder of the build's loop_mix.json)


def meta(text):
    res = {}
    for blk in re.finditer(r"\.name:\s+(_Z\S+)(.*?)(?=\n\s+- \.|\Z)", text, flags=re.S):
        d = {}
        for k in ("vgpr_count", "sgpr_count", "private_segment_fixed_size", "vgpr_spill_count"):
            mm = re.search(r"\." + k + r":\s+(\d+)", blk.group(2))
            if mm:
                d[k] = int(mm.group(1))
        res[blk.group(1)] = d
    return res


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    text = open(path).read()
    md = meta(text)
    for name, body in kernels(text).items():
        if filt not in name:
            continue
        loop = inner_loop(body)
        marks = sum(1 for x in loop if x == "s_setprio")
        ins = [x for x in loop if x != "s_setprio"]
        c = Counter(ins)
        half = sum(v for k, v in c.items() if k in HALF_RATE)
        full = len(ins) - half
        m = md.get(name, {})
        short = re.sub(r"EvNS_8FastArgsEPNS_7PartialE$", "", name)
        print(f"{short:40s} vgpr={m.get('vgpr_count')} sgpr={m.get('sgpr_count')} "
              f"scratch={m.get('private_segment_fixed_size')} loop_valu={len(ins)} half={half} full={full} "
              f"slots={2 * half + full} setprio={marks} "
              f"mix_bound={len(ins) / (2 * max(half, len(ins) / 2)) if ins else 0:.3f}  top={c.most_common(5)}")


if __name__ == "__main__":
    main()
