"""The drop-in `src` package (CPU side): module seam contract, util helpers vs the
reference's golden outputs, and loud failure without a GPU."""
import copy
import json
import os

import numpy as np
import pytest
import torch

from src import util
from src.model import bodypose_25_model, bodypose_model, handpose_model
from islpose import synth

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("name,cls", [("body25", bodypose_25_model), ("coco", bodypose_model),
                                      ("hand", handpose_model)])
def test_state_dict_keys_match_reference(name, cls):
    ref = json.load(open(os.path.join(GOLDEN, "state_dict_keys.json")))[name]
    sd = cls().state_dict()
    assert [[k, list(v.shape)] for k, v in sd.items()] == ref


def test_transfer_roundtrip():
    m = bodypose_25_model()
    w = synth.synth_weights(0)
    sd = util.transfer(m, {k: torch.from_numpy(v) for k, v in w.items()})
    m.load_state_dict(sd)
    assert all(not p.requires_grad for p in m.parameters())
    cw = m.caffe_weights()
    assert set(cw) == set(w)
    assert np.array_equal(cw["Mconv3_stage2_L2_1.weight"].numpy(), w["Mconv3_stage2_L2_1.weight"])
    with pytest.raises(KeyError):
        util.transfer(m, {})


def test_pad_right_down():
    from oracle import cpu_ref
    img = synth.synth_frames(1, 37, 45)[0]
    a, pa = util.padRightDownCorner(img, 8, 128)
    b, pb = cpu_ref.pad_right_down(img)
    assert pa == pb == [0, 0, 3, 3] and np.array_equal(a, b)


def test_npmax_first_max():
    a = np.array([[1.0, 3.0, 3.0], [3.0, 0.0, 3.0]])
    assert util.npmax(a) == (0, 1)


def test_hand_detect_golden():
    z = np.load(os.path.join(GOLDEN, "g5_hand_detect.npz"))
    for c in sorted({k.split("/")[0] for k in z.files}):
        res = util.handDetect(z[c + "/candidate"], z[c + "/subset"], np.zeros(tuple(z[c + "/img_hw"]) + (3,)))
        got = np.array([[x, y, w, int(l)] for x, y, w, l in res], np.int64).reshape(-1, 4)
        assert np.array_equal(got, z[c + "/result"]), c


def test_export_formats_golden():
    g = json.load(open(os.path.join(GOLDEN, "g8_export_formats.json")))
    z = np.load(os.path.join(GOLDEN, "g2_body_post.npz"))
    for case in g["body"]:
        circles, sticks = util.get_bodypose(z[case["case"] + "/candidate"], z[case["case"] + "/subset"],
                                            case["model_type"])
        assert [[float(a), float(b)] for a, b in circles] == case["circles"]
        assert [[float(v) for v in s] for s in sticks] == case["sticks"]
    for h in g["hand"]:
        hands = [np.array(p, np.int64) for p in h["hands"]]
        if h["error"]:
            with pytest.raises(IndexError):
                util.get_handpose(hands)
            continue
        edges, peaks = util.get_handpose(hands)
        assert [[[int(e[0]), [int(v) for v in e[1]], [int(v) for v in e[2]]] for e in hh] for hh in edges] == h["edges"]
        assert [[[int(p[0]), int(p[1]), p[2]] for p in hh] for hh in peaks] == h["peaks"]


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_forward_without_gpu_runs_on_cpu():
    """No visible HIP device: the module runs its own CPU forward (islpose.cpu's net), as the
    reference's model does; a CUDA tensor there is an error."""
    m = handpose_model()
    out = m(torch.zeros(1, 3, 16, 16))
    assert out.shape == (1, 22, 2, 2) and not out.is_cuda


def test_body_constructor_from_weight_file(tmp_path):
    from src.body import Body
    from src.hand import Hand
    p = tmp_path / "body25.pth"
    torch.save({k: torch.from_numpy(v) for k, v in synth.synth_weights(0).items()}, p)
    b = Body(str(p), "body25")
    assert b.njoint == 26 and b.npaf == 52 and b.scale_search == [0.5]
    p2 = tmp_path / "hand.pth"
    torch.save({k: torch.from_numpy(v) for k, v in synth.synth_weights(2).items()}, p2)
    h = Hand(str(p2))
    assert isinstance(h.model, handpose_model)
    c = Body({k: torch.from_numpy(v) for k, v in synth.synth_weights(1).items()}, "xyz")   # falls back to COCO
    assert c.njoint == 19 and isinstance(c.model, bodypose_model)


@pytest.mark.parametrize("cls", [bodypose_25_model, handpose_model])
def test_param_key_sees_every_weight_change(cls):
    """_NativeNet._param_key (what native() compares before re-uploading weights) equals the
    (storage, version) walk over self.parameters() and changes on an in-place edit,
    load_state_dict, a replaced parameter and a replaced top-level child."""
    import torch
    m = cls()
    full = lambda: tuple((p.data_ptr(), p._version) for p in m.parameters())  # noqa: E731
    k0 = m._param_key()
    assert k0 == full()
    with torch.no_grad():
        next(m.parameters()).add_(1.0)
    k1 = m._param_key()
    assert k1 != k0 and k1 == full()
    m.load_state_dict({k: v.clone() for k, v in m.state_dict().items()})
    k2 = m._param_key()
    assert k2 != k1 and k2 == full()
    mod = next(x for x in m.modules() if isinstance(x, torch.nn.Conv2d))
    mod.weight = torch.nn.Parameter(mod.weight.detach().clone())
    k3 = m._param_key()
    assert k3 != k2 and k3 == full()
    name, child = next(iter(m.named_children()))
    setattr(m, name, copy.deepcopy(child))
    k4 = m._param_key()
    assert k4 != k3 and k4 == full()
