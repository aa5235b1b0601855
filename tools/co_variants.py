"""Code-object variants of the product fast_search build for A/Bs through the dev
build's MINEHIP_DEV_CODE_OBJECT hook (round 3):

  padN   N s_nop 0 at every fast_search kernel's entry: the whole kernel body,
         per-nonce loop included, moves by 4N bytes against instruction-cache
         lines (the loop header is not aligned by the compiler)
  cmpH   the per-nonce loop's v_cmp_ge_u32_e32 classed half rate (measured:
         v_cmp_lt_u32_e32 issues at 62 lanes/clk/CU, profiles/r03b_valu_ops.json)
  earlyW the product build (add3 split + issue-priority pass) with the One/Pre Early kernels
         compiled for W waves per SIMD (-DMH_EARLY_WAVES=W; round 5)
  onepreW the same with every One/Pre kernel compiled for W waves (-DMH_ONEPRE_WAVES=W)
  thinN  the product build with a priority marker only where the VALU run it starts is at least N
         instructions long (shorter runs keep the priority they follow): fewer s_setprio per nonce

  python tools/co_variants.py pad0 pad1 pad4 cmpH   # -> build/ab/<variant>.hsaco
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bitcoin-miner_amd", "csrc"))
import issue_prio  # noqa: E402
import valu_rates  # noqa: E402

LLVM = "/opt/rocm/lib/llvm/bin"


def assemble(text, out):
    s = out[:-6] + ".s"
    open(s, "w").write(text)
    o = out[:-6] + ".o"
    subprocess.run([f"{LLVM}/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c",
                    "-o", o, s], check=True)
    subprocess.run([f"{LLVM}/ld.lld", "-shared", "-o", out, o], check=True)


def pad(text, n):
    return re.sub(r"^(_ZN2mh11fast_search\S+:.*)$", lambda m: m.group(1) + "\n" + "\ts_nop 0\n" * n,
                  text, flags=re.M)


def thin_annotate(text, min_run):
    """issue_prio.annotate, but a class change emits its marker only when the run of same-class
    VALU instructions it starts (within the block) is at least min_run long."""
    lines = text.split("\n")
    cls = [issue_prio.valu_class(l) for l in lines]
    out, n, cur, in_kernel = [], 0, None, False
    for k, line in enumerate(lines):
        if re.match(r"^_Z\S+:", line):
            in_kernel, cur = True, None
        elif line.startswith(".Lfunc_end"):
            in_kernel = False
        elif re.match(r"^\.LBB\w*:", line):
            cur = None
        c = cls[k]
        if in_kernel and c is not None and c != cur:
            run = 0
            for j in range(k, len(lines)):
                if re.match(r"^\.LBB\w*:", lines[j]) and j > k:
                    break
                if cls[j] is None:
                    continue
                if cls[j] != c:
                    break
                run += 1
            if cur is None or run >= min_run:
                out.append(f"\ts_setprio {issue_prio.PRIO_HALF if c == 'H' else issue_prio.PRIO_FULL}")
                n += 1
                cur = c
        out.append(line)
    return "\n".join(out), n


def main():
    src = open(os.path.join(ROOT, "build", "fast_search.s")).read()
    src_prod = src
    os.makedirs(os.path.join(ROOT, "build", "ab"), exist_ok=True)
    for v in sys.argv[1:]:
        out = os.path.join(ROOT, "build", "ab", v + ".hsaco")
        if v.startswith("pad"):
            text, _ = issue_prio.annotate(src)
            text = pad(text, int(v[3:]))
        elif v.startswith(("early", "onepre")):
            import add3_split
            s = os.path.join(ROOT, "build", "ab", v + "_src.s")
            macro = "MH_EARLY_WAVES" if v.startswith("early") else "MH_ONEPRE_WAVES"
            subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                            f"-D{macro}={int(v.lstrip('abcdefghijklmnopqrstuvwxyz'))}", "--cuda-device-only", "-S", "-o", s,
                            os.path.join(ROOT, "bitcoin-miner_amd", "csrc", "fast_search.hip")], check=True)
            text, _ = issue_prio.annotate(add3_split.split(open(s).read(), 3)[0])
        elif v.startswith("thin"):
            import add3_split
            text, _ = thin_annotate(add3_split.split(src_prod, 3)[0], int(v[4:]))
        elif v == "cmpH":
            cmps = {o for o in valu_rates.FULL if o.startswith("v_cmp_")}
            old = valu_rates.FULL, valu_rates.HALF
            issue_prio.valu_rate.__globals__["FULL"] = valu_rates.FULL - cmps
            issue_prio.valu_rate.__globals__["HALF"] = valu_rates.HALF | cmps
            try:
                text, _ = issue_prio.annotate(src)
            finally:
                issue_prio.valu_rate.__globals__["FULL"], issue_prio.valu_rate.__globals__["HALF"] = old
        else:
            sys.exit(f"unknown variant {v}")
        assemble(text, out)
        print(out)


if __name__ == "__main__":
    main()
