"""CPU-side checks of the C-ABI library: it loads and exports every symbol that
include/islpose.h declares (no compute calls -- there is no GPU here)."""
import ctypes
import os
import re

import pytest

from islpose import runtime as rt
from islpose import netspec

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    text = open(os.path.join(REPO, "include", "islpose.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(isl_\w+)\s*\(", text, re.M)))


def test_header_symbols_are_exported():
    if not os.path.exists(rt.LIB_PATH):
        pytest.skip("libislpose.so not built")
    lib = ctypes.CDLL(rt.LIB_PATH)
    syms = _header_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(rt.EXPORTS) == syms


def test_param_table_matches_netspec():
    """The native layer tables name exactly the parameters of src/model.py."""
    if not os.path.exists(rt.LIB_PATH):
        pytest.skip("libislpose.so not built")
    for kind in (0, 1, 2):
        net = rt.Net(kind)          # isl_net_create does not touch the device
        assert net.param_names() == [(n, int(__import__("numpy").prod(s))) for n, s in netspec.param_shapes(kind)]


def test_unknown_param_raises_keyerror():
    if not os.path.exists(rt.LIB_PATH):
        pytest.skip("libislpose.so not built")
    import numpy as np
    net = rt.Net(0)
    a = np.zeros(3, np.float32)
    with pytest.raises(KeyError):
        rt.check(rt.lib().isl_net_set_param(net.h, b"no_such_layer.weight", a.ctypes.data_as(ctypes.c_void_p), 3))
    with pytest.raises(KeyError):          # wrong numel
        rt.check(rt.lib().isl_net_set_param(net.h, b"conv1_1.bias", a.ctypes.data_as(ctypes.c_void_p), 3))


def test_body_layout():
    if not os.path.exists(rt.LIB_PATH):
        pytest.skip("libislpose.so not built")
    caps = rt.IslCaps(16, 64, 16, 8)
    lay = rt.body_layout(rt.ISL_BODY25, caps)
    assert lay.peaks % 8 == 0 and lay.record_bytes % 8 == 0
    assert lay.subset + 8 * 27 * 8 <= lay.record_bytes
    assert lay.conns - lay.peaks == 25 * 16 * 3 * 8


def test_new_entry_points_reject_bad_arguments():
    """The batched / pipelined entry points fail with ISL_E_ARG before any device work:
    NULL net or buffers, an empty crop list, a crop of the wrong net (a body net)."""
    if not os.path.exists(rt.LIB_PATH):
        pytest.skip("libislpose.so not built")
    L = rt.lib()
    vp = ctypes.c_void_p
    ws = (ctypes.c_int32 * 1)(100)
    g = (rt.IslScaleGeom * 1)(rt.IslScaleGeom(184, 184, 184, 184))
    hp = (vp * 1)(vp(16))
    assert L.isl_hand_post_crops(None, 1, ws, 1, g, hp, vp(16), None) == rt.ISL_E_ARG
    body = rt.Net(rt.ISL_BODY25)
    assert L.isl_hand_post_crops(body.h, 0, ws, 1, g, hp, vp(16), None) == rt.ISL_E_ARG
    assert L.isl_hand_post_crops(body.h, 1, ws, 1, g, hp, vp(16), None) == rt.ISL_E_ARG   # not a hand net
    assert L.isl_net_check_async(None, vp(16), None) == rt.ISL_E_ARG
    assert L.isl_net_check_async(body.h, None, None) == rt.ISL_E_ARG
    assert L.isl_debug_np_sum(None, 8, vp(16), None) == rt.ISL_E_ARG
    assert L.isl_debug_np_sum(vp(16), 0, vp(16), None) == rt.ISL_E_ARG
