"""Every A/B recipe under tools/ab/ (the experiments behind DESIGN.md / HISTORY.md) loads and
expands into kbench commands (no GPU: --dry-run)."""
import glob
import os
import sys

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import ab  # noqa: E402


def test_recipes_expand():
    recipes = sorted(glob.glob(os.path.join(ROOT, "tools", "ab", "*.json")))
    assert len(recipes) >= 20
    for path in recipes:
        recipe, variants = ab.load(path)
        cmds = ab.commands(recipe, variants)
        assert len(cmds) == len(recipe["workloads"]) and recipe.get("about"), path
        for name, argv in cmds:
            msg, lo, count = ab.WORKLOADS[name]
            assert argv[argv.index("--lo") + 1] == str(lo) and argv.count("--var") == len(variants)
