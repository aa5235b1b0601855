"""One A/B driver for every kernel / plan experiment: a recipe names the variants (environment
settings of the planner knobs, or MINEHIP_DEV_CODE_OBJECT code objects for the dev build) and
the workloads; each workload is one tools/kbench.py process that interleaves the variants round
by round, so an A/B shares one box and one clock.  Run on the GPU box:

  python tools/ab.py tools/ab/<recipe>.json [--tag r04x] [--only d10,cfg1] [--dry-run]

writes gpurun_out/<tag>/kbench_<workload>.json (+ .err) and stops at the first failing step
(a GPU fault, abort or time limit ends the session: nothing more runs on the GPU).

Recipe (JSON):
  {"about": "...", "tag": "r03u",
   "variants": {"name": "K=V,K=V" | "", ...},          # "" = the product build as is
   "code_objects": {"name": "build/ab/x.hsaco"},       # shorthand: MINEHIP_DEV_CODE_OBJECT=...
   "workloads": [["d10", 7, "clock"], ["cfg1", 9], ...],  # WORKLOADS name, rounds, optional clock,
                                                          # optional "energy<R>" (R energy windows)
   "retired": "why"}   # optional: the knobs it varies left the library; kept as the record, not run
The recipes under tools/ab/ are the experiments behind DESIGN.md and profiles/ (HISTORY.md).
"""
import argparse
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# name -> (message, first nonce, nonces): BASELINE workloads and the buckets the A/Bs isolate
WORKLOADS = {
    "d10": ("cmu440", 10 ** 9, 1 << 32),                  # configs[1]'s d = 10 bucket layout, <4, One>
    "d9": ("cmu440", 10 ** 8, 9 * 10 ** 8),               # d = 9, <3, One>
    "d79": ("cmu440", 10 ** 6, 999 * 10 ** 6),            # d = 7..9
    "cfg1": ("cmu440", 0, 1 << 32),                       # BASELINE configs[1], whole
    "cfg3a": ("a" * 100, 0, 1 << 34),                     # configs[2]: host midstate block
    "cfg3b": ("x" * 60, 0, 1 << 34),                      # configs[2]: two tail blocks
    "cfg4slice": ("cmu440", 1 << 39, 1 << 36),            # a 2^36 slice of configs[3]
    "cfg4step": ("cmu440", 1 << 39, (1 << 40) // 20),     # one of configs[3]'s 20 bench steps
    "shard8": ("cmu440", 1 << 39, 6871947673),            # one 8-GPU shard of a configs[3] step
    "shard4": ("cmu440", 1 << 39, 13743895347),           # one 4-GPU shard
    "shard2": ("cmu440", 1 << 39, 27487790694),           # one 2-GPU shard
    "p55": (("cmu440-" * 10)[:55], 0, 1 << 32),           # <13|14|15, Two> layouts
    # round 5: fixtures whose d = 10 bucket takes an Early layout (fast_search<J, 3..5>)
    "one10": (("cmu440-" * 10)[:30], 0, 1 << 32),         # <9, One> -> <8, OneEarly>
    "two14": (("cmu440-" * 10)[:48], 0, 1 << 32),         # <14, Two> -> <13, TwoEarly>
    "pre2": (("cmu440-" * 10)[:62], 0, 1 << 32),          # d = 9: <1, Pre> -> <0, PreEarly>
    # ... and one bucket of each, alone
    "x60d10": ("x" * 60, 10 ** 9, 1 << 33),               # <1, Pre> -> <0, PreEarly>, p = 3
    "x60d11": ("x" * 60, 10 ** 10, 1 << 33),              # <1, Pre> -> <0, PreEarly>, p = 4
    "one10d9": (("cmu440-" * 10)[:30], 10 ** 8, 9 * 10 ** 8),   # <9, One> -> <8, OneEarly>
    "two14d10": (("cmu440-" * 10)[:48], 10 ** 9, 1 << 32),      # <14, Two> -> <13, TwoEarly>
    "a100d10": ("a" * 100, 10 ** 9, 1 << 33),             # configs[2]'s 100 x 'a' d = 10 bucket, <11, One>
    "one10d10": (("cmu440-" * 10)[:30], 10 ** 9, 1 << 32),      # <10, One>
    "one8": (("cmu440-" * 10)[:25], 0, 1 << 32),          # <7|8, One>
}
FATAL = {124, 134, 137, 139}


def load(path):
    with open(path) as f:
        r = json.load(f)
    variants = dict(r.get("variants", {}))
    for name, co in r.get("code_objects", {}).items():
        variants[name] = f"MINEHIP_DEV_CODE_OBJECT={co}"
    if not variants or not r.get("workloads"):
        raise SystemExit(f"{path}: a recipe needs variants and workloads")
    # kbench.py reads a variant as comma-separated K=V settings; anything else would reach the
    # library as part of one value (round 5 found r04_fuse_tail's "A=1 B=2" variants set only A)
    for name, env in variants.items():
        for kv in filter(None, env.split(",")):
            if not re.fullmatch(r"MINEHIP_\w+=[^\s=]*", kv) and not r.get("retired"):
                raise SystemExit(f"{path}: variant {name!r}: {kv!r} is not one MINEHIP_*=value setting")
    for w in r["workloads"]:
        if w[0] not in WORKLOADS:
            raise SystemExit(f"{path}: unknown workload {w[0]!r} (known: {', '.join(WORKLOADS)})")
    return r, variants


def commands(recipe, variants, only=None):
    """[(workload name, argv)] of the kbench processes a recipe runs."""
    out = []
    for w in recipe["workloads"]:
        name, rounds = w[0], int(w[1])
        if only and name not in only:
            continue
        msg, lo, count = WORKLOADS[name]
        argv = [sys.executable, os.path.join(ROOT, "tools", "kbench.py"), "--msg", msg, "--lo", str(lo),
                "--count", str(count), "--rounds", str(rounds)]
        if "clock" in w[2:]:
            argv.append("--clock")
        for opt in w[2:]:  # "energy<R>": R interleaved clock + energy windows per variant (kbench --energy)
            if isinstance(opt, str) and opt.startswith("energy"):
                argv += ["--energy", opt[len("energy"):] or "3"]
        for v, env in variants.items():
            argv += ["--var", f"{v}:{env}"]
        out.append((name, argv))
    return out


def ensure_code_objects(recipe):
    """Build the recipe's missing code objects where the run happens (the
    variants are not pushed to every GPU box): build/isa/<v>.hsaco by tools/isa_variant.py <v>,
    build/ab/<v>.hsaco by tools/co_variants.py <v> (from the compiler's build/fast_search.s)."""
    for name, co in recipe.get("code_objects", {}).items():
        path = os.path.join(ROOT, co)
        if os.path.exists(path):
            continue
        d, v = os.path.dirname(co), os.path.basename(co)[:-len(".hsaco")]
        if d == "build/isa":
            cmd = [sys.executable, os.path.join(ROOT, "tools", "isa_variant.py"), v]
        elif d == "build/ab":
            s = os.path.join(ROOT, "build", "fast_search.s")
            if not os.path.exists(s):
                subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                                "--cuda-device-only", "-S", "-o", s,
                                os.path.join(ROOT, "bitcoin-miner_amd", "csrc", "fast_search.hip")], check=True)
            cmd = [sys.executable, os.path.join(ROOT, "tools", "co_variants.py"), v]
        else:
            raise SystemExit(f"code object {co} ({name}) is missing and has no builder")
        print(f"building {co}: {' '.join(cmd[1:])}", flush=True)
        if subprocess.run(cmd, cwd=ROOT).returncode != 0 or not os.path.exists(path):
            raise SystemExit(f"could not build {co}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("recipe")
    ap.add_argument("--tag", default=None, help="output directory under gpurun_out/ (default: the recipe's)")
    ap.add_argument("--only", default=None, help="comma-separated workloads to run")
    ap.add_argument("--timeout", type=int, default=400, help="seconds per kbench process")
    ap.add_argument("--dry-run", action="store_true")
    a = ap.parse_args()
    recipe, variants = load(a.recipe)
    if recipe.get("retired") and not a.dry_run:
        raise SystemExit(f"{a.recipe}: retired ({recipe['retired']})")
    out = os.path.join(ROOT, "gpurun_out", a.tag or recipe.get("tag", "ab"))
    cmds = commands(recipe, variants, set(a.only.split(",")) if a.only else None)
    if a.dry_run:
        for name, argv in cmds:
            print(name, " ".join(argv[1:]))
        return
    os.makedirs(out, exist_ok=True)
    ensure_code_objects(recipe)
    for name, argv in cmds:
        with open(os.path.join(out, f"kbench_{name}.json"), "w") as fo, \
                open(os.path.join(out, f"kbench_{name}.err"), "w") as fe:
            try:
                rc = subprocess.run(["timeout", "-k", "10", str(a.timeout), *argv], stdout=fo, stderr=fe).returncode
            except KeyboardInterrupt:
                raise SystemExit(130)
        print(f"{name}: rc={rc}", flush=True)
        with open(os.path.join(out, f"kbench_{name}.json")) as f:
            print(f.read().strip(), flush=True)
        if rc != 0:
            raise SystemExit(rc if rc in FATAL or rc > 128 else 1)


if __name__ == "__main__":
    main()
