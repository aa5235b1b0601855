"""Build gfx950 code objects of search_kernels.hip with hand-edited ISA, for
A/B runs through the dev build's MINEHIP_DEV_CODE_OBJECT hook (`make dev`; experiments
only).

  python tools/isa_variant.py base e64      # -> build/isa/<variant>.hsaco (from fast_search.hip)
  python tools/kbench.py --var base:MINEHIP_DEV_CODE_OBJECT=build/isa/base.hsaco \
                         --var e64:MINEHIP_DEV_CODE_OBJECT=build/isa/e64.hsaco

Variants (edits apply inside the fast_search kernels only):
  base  the compiler's assembly, re-assembled unchanged: the kernels WITHOUT the
        issue-priority pass the library's own build applies
  prio  the library's build (bitcoin-miner_amd/csrc/issue_prio.py), re-made here
  e64   every VOP2 v_add_u32 / v_lshrrev_b32 without a literal operand in its
        VOP3 (_e64) encoding: same operation, other encoding.  The r02e probes
        (tools/gen_valu_pair.py) show a VOP3 full-rate op after a half-rate
        one co-issuing where a VOP2 one does not (HF3 3.74 vs HF 4.03 cycles).
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "bitcoin-miner_amd", "csrc")
OUT = os.path.join(ROOT, "build", "isa")
HIPCC = "/opt/rocm/bin/hipcc"
LLVM = "/opt/rocm/lib/llvm/bin"
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950"]


def compile_s(path, extra=()):
    subprocess.run([HIPCC, *FLAGS, *extra, "--cuda-device-only", "-S", "-o", path,
                    os.path.join(CSRC, "fast_search.hip")], check=True)


def assemble(s_path, co_path):
    o_path = co_path[:-6] + ".o"
    subprocess.run([f"{LLVM}/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c",
                    s_path, "-o", o_path], check=True)
    subprocess.run([f"{LLVM}/ld.lld", "-shared", o_path, "-o", co_path], check=True)


INLINE = re.compile(r"^-?\d+$")


def is_inline(op):
    op = op.strip()
    if op.startswith(("v", "s", "vcc", "exec", "m0")) and not op.startswith("0x"):
        return True
    if INLINE.match(op):
        return -16 <= int(op) <= 64
    return False


def to_e64(line, ops=("v_add_u32", "v_lshrrev_b32")):
    m = re.match(r"^(\s+)(" + "|".join(ops) + r")_e32\s+(.*)$", line)
    if not m:
        return line, False
    args = [a.strip() for a in m.group(3).split(",")]
    if not all(is_inline(a) for a in args[1:]):
        return line, False  # gfx9 VOP3 takes no literal
    return f"{m.group(1)}{m.group(2)}_e64 {', '.join(args)}", True


def in_fast(text):
    """Yield (line, inside a fast_search function body)."""
    inside = False
    for line in text.split("\n"):
        if re.match(r"^_ZN2mh11fast_search\S*:", line):
            inside = True
        elif inside and (line.startswith(".Lfunc_end") or "s_endpgm" in line):
            yield line, True
            inside = False
            continue
        yield line, inside


# source-level variants: the kernel source compiled with extra defines
DEFINES = {  # name: (extra compiler flags, apply the issue-priority pass)
    # (the s_barrier variants sync1/sync10 of round 2, -4%, profiles/r02k_kbench_sync.json, were removed
    # from the kernel source in round 3)
    "prio_w8": (["-DMH_MIN_WAVES=8"], True),   # <= 64 VGPRs: 8 waves/SIMD
    "split_w8": (["-DMH_MIN_WAVES=8"], "split"),  # the same with the build's add3 split
    "split_w1": (["-DMH_MIN_WAVES=1"], "split"),  # no register cap: the allocator's own choice
    "prio_w6": (["-DMH_MIN_WAVES=6"], True),
    "prio_ilp": (["-mllvm", "--amdgpu-sched-strategy=iterative-ilp"], True),
    "prio_maxilp": (["-mllvm", "--amdgpu-sched-strategy=max-ilp"], True),
    "grp_maxilp": (["-mllvm", "--amdgpu-sched-strategy=max-ilp"], "sched"),   # more VGPRs, then grouping
    "grp_ilp": (["-mllvm", "--amdgpu-sched-strategy=iterative-ilp"], "sched"),
    # timing-only upper bounds (WRONG results): grouping with register dependencies ignored
    "ub_grp_ilp": (["-mllvm", "--amdgpu-sched-strategy=iterative-ilp"], "ub"),
    "ub_grp_def": ([], "ub"),
}


def variant(name, base_text):
    if name == "base":
        return base_text, 0
    if name == "e64":
        out, n = [], 0
        for line, fast in in_fast(base_text):
            if fast:
                line, ch = to_e64(line)
                n += ch
            out.append(line)
        return "\n".join(out), n
    if name.startswith("a3pat"):
        # a3pat<pattern>: the add3 split at the '1's of a 0/1 pattern repeated over each fast
        # kernel's add3s (a3pat001 = a3split3 = the build), then the issue-priority pass
        t, n = add3_split.split(base_text, 0, pattern=name[len("a3pat"):])
        t2, n2 = prio_phases(t)
        return t2, n + n2
    if name.startswith("a3far"):
        # a3far<pct>: split the pct% of each fast kernel's add3s whose results are read latest
        t, n = add3_split.split_by_slack(base_text, int(name[len("a3far"):]) / 100)
        t2, n2 = prio_phases(t)
        return t2, n + n2
    if name.startswith("a3split"):
        # a3split<k>: every k-th v_add3_u32 of the fast kernels as two full-rate adds, then the
        # issue-priority pass.  A half-rate op cannot share its quad-cycle with another half-rate
        # op, so the loop needs >= max(H, N/2) quad-cycles; trading some add3 (1 H) for two adds
        # (2 F) lowers H below N/2's growth (J = 4: H 701, N 1196).
        k = int(name[len("a3split"):])
        t, n = add3_split.split(base_text, k)  # the build's own pass (per-kernel count)
        t2, n2 = prio_phases(t)
        return t2, n + n2
    if name.startswith("sched_"):
        # sched_<D>_<R>: tools/sched_pass.py grouping, then the issue-priority pass
        from sched_pass import reorder
        _, dd, rr = name.split("_")
        t, nb = reorder(base_text, D=int(dd), R=int(rr))
        t2, n2 = prio_phases(t)
        return t2, n2
    if name.startswith("pv_"):
        # pv_<minF>_<leadF>_<leadH>: marker-placement variants of the issue-priority pass
        _, mf, lf, lh = name.split("_")
        return prio_variant(base_text, int(mf), int(lf), int(lh))
    if name.startswith("dup"):
        # dup<k>: the product build with every k-th s_setprio written twice.  The copy changes
        # nothing the wave does (same priority) but adds 4 bytes of code: a probe of whether
        # instruction fetch (32-byte requests per wave from the I-cache shared by two CUs)
        # co-limits the loop.
        k = int(name[3:])
        t, _ = prio_phases(base_text)
        out, n, i = [], 0, 0
        for line, fast in in_fast(t):
            out.append(line)
            if fast and re.match(r"^\s+s_setprio\s+\d+\s*$", line):
                i += 1
                if i % k == 0:
                    out.append(line)
                    n += 1
        return "\n".join(out), n
    if name.startswith("prio"):
        return prio_phases(base_text)
    raise SystemExit(f"unknown variant {name}")


sys.path.insert(0, CSRC)
from issue_prio import annotate, valu_class  # noqa: E402
import add3_split  # noqa: E402


def is_vgpr(op):
    return re.match(r"^v\d+$", op) is not None


def prio_phases(text):
    return annotate(text)


def prio_variant(text, min_f, lead_f, lead_h):
    """Issue-priority markers with (a) full-rate runs shorter than min_f left at priority 3 and
    (b) each marker moved lead_f / lead_h VALU instructions earlier (the wave yields, or reclaims,
    before its head changes class).  Blocks are handled separately (a branch may enter a label)."""
    lines = text.split("\n")
    out_marks = {}  # line index -> marker text inserted before it
    n = 0
    block = []      # (line index, class) of the current block's VALU instructions

    def flush():
        nonlocal n
        if not block:
            return
        cls = [c for _, c in block]
        # runs
        runs, i = [], 0
        while i < len(cls):
            j = i
            while j < len(cls) and cls[j] == cls[i]:
                j += 1
            runs.append([cls[i], i, j])
            i = j
        for r in runs:  # short full-rate runs stay in the surrounding half-rate phase
            if r[0] == "F" and r[2] - r[1] < min_f and len(runs) > 1:
                r[0] = "H"
        merged = []
        for r in runs:
            if merged and merged[-1][0] == r[0]:
                merged[-1][2] = r[2]
            else:
                merged.append(r)
        prev_start = -1
        for c, a, _ in merged:
            lead = lead_f if c == "F" else lead_h
            pos = max(prev_start + 1, a - lead) if a > 0 else 0
            prev_start = pos
            out_marks[block[pos][0]] = f"\ts_setprio {3 if c == 'H' else 0}"
            n += 1

    in_kernel = False
    for k, line in enumerate(lines):
        if re.match(r"^_Z\S+:", line):
            flush(); block = []; in_kernel = True
        elif line.startswith(".Lfunc_end"):
            flush(); block = []; in_kernel = False
        elif re.match(r"^\.LBB\w*:", line):
            flush(); block = []
        if in_kernel:
            c = valu_class(line)
            if c is not None:
                block.append((k, c))
    flush()
    out = []
    for k, line in enumerate(lines):
        if k in out_marks:
            out.append(out_marks[k])
        out.append(line)
    return "\n".join(out), n


def main():
    os.makedirs(OUT, exist_ok=True)
    base_s = os.path.join(OUT, "base.s")
    compile_s(base_s)
    text = open(base_s).read()
    for name in sys.argv[1:] or ["base", "e64"]:
        s_path = os.path.join(OUT, f"{name}.s")
        if name in DEFINES:
            flags, prio = DEFINES[name]
            compile_s(s_path, flags)
            n = 0
            if prio in ("sched", "ub"):
                from sched_pass import reorder
                t, _ = reorder(open(s_path).read(), D=1, R=99, raw_only=(prio == "ub"))
                t, n = prio_phases(t)
                open(s_path, "w").write(t)
            elif prio == "split":
                t, _ = add3_split.split(open(s_path).read(), 3)
                t, n = prio_phases(t)
                open(s_path, "w").write(t)
            elif prio:
                t, n = prio_phases(open(s_path).read())
                open(s_path, "w").write(t)
        else:
            t, n = variant(name, text)
            if name != "base":
                open(s_path, "w").write(t)
        assemble(s_path, os.path.join(OUT, f"{name}.hsaco"))
        print(f"{name}: {n} instructions edited -> build/isa/{name}.hsaco")


if __name__ == "__main__":
    main()
