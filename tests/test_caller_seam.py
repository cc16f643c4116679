"""The caller seam of the north star: the reference's scripts (extract_features*.py,
demo_isl_translate*.py, the demos) import ``src`` names; every one must resolve with
this repository's ``src`` in place -- replaced modules from here, the rest through the
fall-through to the reference's original ``src`` (src/__init__.py).  The import lines
come from tests/golden/caller_imports.json (an ast scan of the reference scripts by
tests/golden/make_caller_imports.py); no reference script is executed."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "isl-signlanguage-translation_amd")
FIX = json.load(open(os.path.join(REPO, "tests", "golden", "caller_imports.json")))
NORTH_STAR = ("extract_features.py", "extract_features_mp.py", "extract_featuressingle.py",
              "demo_isl_translate.py", "demo_isl_translate_one_model.py")


def _replaced():
    return {os.path.splitext(f)[0] for f in os.listdir(os.path.join(PKG, "src")) if f.endswith(".py")}


def _imports(scripts=None):
    for script, imps in FIX["scripts"].items():
        if scripts is None or script in scripts:
            for e in imps:
                yield script, e


def test_fixture_covers_the_north_star_scripts():
    assert set(NORTH_STAR) <= set(FIX["scripts"])


def test_replaced_modules_export_every_imported_name():
    """`from src.X import Y` with X replaced here: Y exists in our module."""
    import importlib
    replaced = _replaced()
    seen = 0
    for script, e in _imports():
        mod = e["module"]
        if mod == "src":
            for n in e["names"]:
                assert n in replaced or n in FIX["reference_src_modules"], (script, e)
            continue
        top = mod.split(".")[1]
        if top not in replaced:
            continue
        m = importlib.import_module(mod)
        for n in e["names"]:
            assert hasattr(m, n), (script, e["line"], mod, n)
            seen += 1
    assert seen >= 8


def test_other_modules_fall_through_to_reference_src(tmp_path):
    """Everything not replaced is a module of the reference's own src (fall-through),
    and the fall-through works in the symlink layout INTEGRATION.md recommends: a
    script next to ``src -> <this repo>/src`` with the original kept as ``src.orig``
    imports every name the reference scripts import (stub originals here)."""
    replaced = _replaced()
    fall = {}
    for script, e in _imports():
        if e["module"] == "src":
            continue
        top = e["module"].split(".")[1]
        if top not in replaced:
            assert top in FIX["reference_src_modules"] or top == "keras", e
            fall.setdefault(e["module"], set()).update(e["names"])
    assert "src.expression_mapping" in fall
    ref = tmp_path / "ref"
    orig = ref / "src.orig"
    (orig / "keras").mkdir(parents=True)
    (orig / "__init__.py").write_text("")
    (orig / "keras" / "__init__.py").write_text("")
    for mod, names in fall.items():
        path = orig.joinpath(*mod.split(".")[1:]).with_suffix(".py")
        path.write_text("".join("%s = %r\n" % (n, n) for n in sorted(names)) or "ORIGINAL = True\n")
    # the reference's util.py carries the drawing helpers the drop-in delegates to
    (orig / "util.py").write_text("def drawStickmodel(img, *a):\n    return ('drawn', img)\n")
    for m in ("model.py", "body.py", "hand.py", "ISL_Model_parameter.py"):   # the reference's marker files
        if not (orig / m).exists():
            (orig / m).write_text("ORIGINAL = True\n")
    os.symlink(os.path.join(PKG, "src"), ref / "src")
    lines = ["import sys", "sys.path.insert(0, %r)" % str(ref)]
    for script, e in _imports():
        if e["names"]:
            lines.append("from %s import %s" % (e["module"], ", ".join(e["names"])))
        else:
            lines.append("import %s" % e["module"])
    lines += ["import src, src.util",
              "assert src.util.drawStickmodel('frame', 1, 2, 3, 4) == ('drawn', 'frame')",
              "assert expression_mapping == 'expression_mapping'",
              "assert src.__path__[-1].endswith('src.orig')",
              "print('ok')"]
    (ref / "check.py").write_text("\n".join(lines) + "\n")
    env = {k: v for k, v in os.environ.items() if k != "ISLPOSE_REFERENCE_SRC"}
    env["PYTHONPATH"] = ""
    r = subprocess.run([sys.executable, str(ref / "check.py")], cwd=str(ref), env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr


def test_drawing_without_reference_raises(monkeypatch):
    from src import util
    monkeypatch.setattr(util, "reference_util", lambda: None)
    with pytest.raises(NotImplementedError):
        util.drawStickmodel(None, [], [], [], [])


def test_isl_sign_pos_to_returns_self_and_pins_device():
    """extract_features_mp.py:150: ``model = model.to(device)``."""
    from src.ISL_Model_parameter import ISLSignPos, ISLSignPosTranslator
    m = ISLSignPos(None, None)
    assert m.to(torch.device("cuda:1")) is m and m._device == 1
    assert m.to("cpu") is m and m._device == 1
    t = ISLSignPosTranslator(None, None, lambda x: x)
    assert t.to("cuda:0") is t and t._device == 0


def test_translator_cache_dropped_when_weights_change():
    """Feature rows cached for a rolling window are recomputed after the nets'
    weights change (load_state_dict copies in place: the parameter versions move)."""
    from src.ISL_Model_parameter import ISLSignPosTranslator
    body, hand = torch.nn.Linear(2, 2), torch.nn.Linear(2, 2)
    t = ISLSignPosTranslator(body, hand, lambda x: np.asarray(x).sum())
    counted = []

    def fake(frames):
        counted.append(len(frames))
        out = []
        for f in frames:
            cand = np.array([[float(f[0, 0, 0]), 1.0, 0.9, 0.0]])
            subset = np.full((1, 27), -1.0)
            subset[0, 0], subset[0, -2], subset[0, -1] = 0, 0.9, 1
            out.append((cand, subset, []))
        return out
    t.call_batch = fake
    frames = np.zeros((21, 4, 4, 3), np.uint8)
    frames[:, 0, 0, 0] = np.arange(21)
    t.call(frames[:20])
    t.call(frames[1:21])
    assert counted == [20, 1]
    with torch.no_grad():
        body.weight.copy_(body.weight + 1)
    t.call(frames[1:21])
    assert counted == [20, 1, 20]


def test_fall_through_ignores_unrelated_src(tmp_path, monkeypatch):
    """A ``src`` package on sys.path without the reference's files (model.py, body.py,
    hand.py, util.py, ISL_Model_parameter.py) never becomes the fall-through."""
    import sys
    import src
    other = tmp_path / "src"
    other.mkdir()
    (other / "__init__.py").write_text("")
    (other / "util.py").write_text("raise SystemExit('must not be imported')\n")
    monkeypatch.delenv("ISLPOSE_REFERENCE_SRC", raising=False)
    monkeypatch.setattr(sys, "path", [str(tmp_path)] + list(sys.path))
    assert src.reference_src() != str(other)
    for m in src._MARKERS:
        (other / m).write_text("")
    assert src.reference_src() == str(other)
