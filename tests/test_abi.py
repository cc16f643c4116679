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


def test_lane_assign_hand_and_pyramid_scales():
    """rt.lane_assign (the streams of a pyramid's scales): the hand's four crop scales
    (184/368/552/736 px) -> [736] [552] [368 then 184] on three lanes, largest enqueued
    first; colliding sizes share a lane in their order; fewer sizes than lanes use fewer."""
    keys = [(184, 184), (368, 368), (552, 552), (736, 736)]
    lane, order, n = rt.lane_assign(keys, 3)
    assert n == 3 and order == [3, 2, 1, 0]
    assert lane[3] != lane[2] and lane[1] == lane[0] and len({lane[3], lane[2], lane[1]}) == 3
    body = [(192, 336), (192, 336), (368, 656)]      # two scales padding to one size
    lane, order, n = rt.lane_assign(body, 3)
    assert n == 2 and lane[0] == lane[1] != lane[2] and order == [2, 0, 1]
    lane, order, n = rt.lane_assign(keys, 1)
    assert n == 1 and lane == [0, 0, 0, 0]
