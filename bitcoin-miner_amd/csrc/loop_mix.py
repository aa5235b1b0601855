"""loop_mix.py -- the issued instruction mix of every fast_search per-nonce loop (Makefile).

    python3 loop_mix.py build/fast_search_prio.s build/fast_loop_mix.json

The build changes the compiler's instruction stream (add3_split.py turns every third v_add3 into
two full-rate adds), so the loop the GPU runs issues more instructions than the algorithm counts
(plan.cpp nonce_cost) and fewer half-rate ones.  bench.py prices `frac` on the algorithm's count
and takes the bound a build can reach from this file: for each fast_search<J, MODE>, the VALU
instructions and the half-rate ones of its per-nonce loop, read from the assembly that is
assembled into the embedded code object.  tools/isa_report.py prints the same loops.
"""
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from valu_rates import valu_rate  # noqa: E402  (the opcode tables of the issue-priority pass)


def kernels(text):
    """{mangled name: assembly body up to its s_endpgm} for every kernel of the file."""
    out = {}
    for m in re.finditer(r"^(_Z\S+):", text, flags=re.M):
        end = text.find("s_endpgm", m.end())
        out[m.group(1)] = text[m.end():end]
    return out


def loop_blocks(body):
    """Opcodes of every loop-header block (up to its first scalar branch)."""
    lines = body.split("\n")
    out = []
    for i, l in enumerate(lines):
        if "Loop Header" in l:
            ops = []
            for j in range(i, len(lines)):
                s = lines[j].strip()
                if s and not s.startswith((";", ".")):
                    ops.append(s.split()[0])
                if s.startswith("s_cbranch_scc") or s.startswith("s_branch"):
                    break
            out.append(ops)
    return out


def per_nonce_loop(body):
    """All opcodes of the loop block with the most VALU instructions: the per-nonce body of
    fast_search (its innermost loop is the rare candidate scan)."""
    blocks = loop_blocks(body)
    return max(blocks, key=lambda ops: sum(o.startswith("v_") for o in ops)) if blocks else []


def inner_loop(body):
    """Opcodes (VALU and s_setprio) of the per-nonce loop."""
    return [o for o in per_nonce_loop(body) if o.startswith("v_") or o.startswith("s_setprio")]


FAST = re.compile(r"^_ZN2mh11fast_searchILi(\d+)ELi(\d+)EE")


def loop_mix(text):
    """{"J,MODE": {"valu": N, "half": H}} of every fast_search kernel's per-nonce loop."""
    out = {}
    for name, body in kernels(text).items():
        m = FAST.match(name)
        if not m:
            continue
        ins = [x for x in inner_loop(body) if x != "s_setprio"]
        out[f"{m.group(1)},{m.group(2)}"] = {
            "valu": len(ins), "half": sum(1 for x in ins if valu_rate(x) == "H"),
            # private-memory (spill) accesses inside the per-nonce loop: must stay 0
            "loop_spill_ops": sum(1 for o in per_nonce_loop(body) if o.startswith(("scratch_", "buffer_")))}
    return out


def fast_kernels(layout=os.path.join(os.path.dirname(os.path.abspath(__file__)), "layout.hpp")):
    """{(J, MODE)} of layout.hpp's MH_FAST_KERNELS list: the instantiated fast_search layouts."""
    text = open(layout).read()
    body = text[text.index("#define MH_FAST_KERNELS(X)"):]
    body = body[:body.index("\n\n")]
    modes = {m: int(v) for m, v in re.findall(r"(kMode\w+)\s*=\s*(\d+)", text)}
    return {(int(j), modes[m]) for j, m in re.findall(r"X\((\d+),\s*(kMode\w+)\)", body)}


def main():
    src, dst = sys.argv[1], sys.argv[2]
    mix = loop_mix(open(src).read())
    want = {f"{j},{m}" for j, m in fast_kernels()}
    if set(mix) != want or any(v["valu"] == 0 for v in mix.values()):
        sys.exit(f"loop_mix: expected the {len(want)} fast_search loops of layout.hpp in {src}, found {len(mix)}")
    with open(dst, "w") as f:
        json.dump(mix, f, indent=0, sort_keys=True)
    print(f"loop_mix: {len(mix)} per-nonce loops -> {dst}")


if __name__ == "__main__":
    main()
