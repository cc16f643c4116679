"""Drop-in replacement for the reference's ``src`` package (pytorch-openpose core of
ISL-SignLanguage-Translation), backed by libislpose.so on MI355X.

Put ``isl-signlanguage-translation_amd`` on sys.path (ahead of the reference's own
``src``) and the reference scripts' ``from src.body import Body`` /
``from src.hand import Hand`` / ``from src import util`` /
``from src.ISL_Model_parameter import ISLSignPos`` resolve here.
"""
import os as _os
import sys as _sys

_pkg_root = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
if _pkg_root not in _sys.path:
    _sys.path.insert(0, _pkg_root)
