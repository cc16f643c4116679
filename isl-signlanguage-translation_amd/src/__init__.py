"""Drop-in replacement for the reference's ``src`` package (pytorch-openpose core of
ISL-SignLanguage-Translation), backed by libislpose.so on MI355X.

Put ``isl-signlanguage-translation_amd`` on sys.path (ahead of the reference's own
``src``), or symlink this directory in place of the reference's ``src`` (keeping the
original as ``src.orig``), and the reference scripts' ``from src.body import Body`` /
``from src.hand import Hand`` / ``from src import util`` /
``from src.ISL_Model_parameter import ISLSignPos`` resolve here.

Modules this package does not replace -- the ones off the keypoint path, e.g.
``src.expression_mapping`` (demo_isl_translate.py:30) and ``src.dataloader`` --
fall through to the reference's own files: the original ``src`` directory is
appended to this package's ``__path__``, so they import from it unchanged (and
their own ``from src.X import ...`` lines come back here).  The original is looked
up, in order, at ``$ISLPOSE_REFERENCE_SRC``, at ``src.orig`` next to this package
as imported (the symlink layout), and at any other ``src`` directory on sys.path.
"""
import os as _os
import sys as _sys

_here = _os.path.dirname(_os.path.abspath(__file__))     # as imported (a symlink stays a symlink)
_pkg_root = _os.path.dirname(_os.path.realpath(__file__))
_pkg_root = _os.path.dirname(_pkg_root)
if _pkg_root not in _sys.path:
    _sys.path.insert(0, _pkg_root)


# files the reference's src package holds (pytorch-openpose core + the ISL wrapper): a
# candidate found by search must have all of them, so an unrelated project's ``src``
# (the cwd, site-packages) never becomes the fall-through
_MARKERS = ("model.py", "body.py", "hand.py", "util.py", "ISL_Model_parameter.py")


def _is_reference_src(c):
    return all(_os.path.isfile(_os.path.join(c, m)) for m in _MARKERS)


def reference_src():
    """The reference's original ``src`` directory, or None when it cannot be found.
    ``$ISLPOSE_REFERENCE_SRC`` is taken as given; ``src.orig`` next to this package and
    ``src`` directories on sys.path must carry the reference's marker files."""
    real = _os.path.realpath(_here)
    cands = []
    if _os.environ.get("ISLPOSE_REFERENCE_SRC"):
        cands.append((_os.environ["ISLPOSE_REFERENCE_SRC"], False))
    cands.append((_os.path.join(_os.path.dirname(_here), "src.orig"), True))
    for p in _sys.path:
        cands.append((_os.path.join(p or _os.getcwd(), "src"), True))
    for c, need_markers in cands:
        if c and _os.path.isdir(c) and _os.path.realpath(c) != real and \
                _os.path.isfile(_os.path.join(c, "__init__.py")) and (not need_markers or _is_reference_src(c)):
            return c
    return None


_orig = reference_src()
if _orig is not None and _orig not in __path__:
    __path__.append(_orig)
