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


def test_malformed_variant_is_refused(tmp_path):
    """A variant's settings are comma-separated MINEHIP_*=value pairs (kbench.py splits on ','): a
    space-separated pair would reach the library as one value (r04_fuse_tail's 2^27 / 2^29
    variants set only the first), so ab.load refuses it unless the recipe is retired."""
    import json
    import pytest
    bad = {"about": "x", "variants": {"a": "MINEHIP_QUEUE=1 MINEHIP_FINE_TAIL=0"}, "workloads": [["cfg1", 1]]}
    p = tmp_path / "bad.json"
    p.write_text(json.dumps(bad))
    with pytest.raises(SystemExit):
        ab.load(str(p))
    p.write_text(json.dumps(dict(bad, variants={"a": "MINEHIP_QUEUE=1,MINEHIP_FINE_TAIL=0"})))
    assert ab.load(str(p))[1] == {"a": "MINEHIP_QUEUE=1,MINEHIP_FINE_TAIL=0"}
    p.write_text(json.dumps(dict(bad, retired="kept as the record")))
    ab.load(str(p))  # the record of a retired experiment loads as it ran
