"""Drop-in for the reference's src/model.py (module seam).

``bodypose_25_model``, ``bodypose_model`` and ``handpose_model`` are nn.Modules
whose parameters carry exactly the reference's state_dict keys (so
``load_state_dict(util.transfer(model, torch.load(path)))`` works unchanged,
model.py:66-407 / util.py:35-44), but whose ``forward`` runs the network in
libislpose.so (FP32-MFMA HIP kernels).  Parameters are pushed to the native
net on first use and whenever they change.

Without a visible HIP device forward runs the modules themselves on the CPU in the
reference's dataflow (``cpu_forward``; model.py:171-207, 301-328, 394-407) -- the GPU-less
path of src/body.py / src/hand.py (islpose.cpu).  With a device it never falls back.
"""
from __future__ import annotations

from collections import OrderedDict

import torch
import torch.nn as nn

from islpose import netspec
from islpose import runtime as rt


def caffe_name(state_key: str) -> str:
    """util.transfer's key mapping (util.py:37-43): drop 3 leading components for
    body_25's nested Mconv blocks (> 4 components), else 1."""
    parts = state_key.split(".")
    return ".".join(parts[3:]) if len(parts) > 4 else ".".join(parts[1:])


def _conv_layers(specs, pools_after=()):
    """[(name, module)] for a make_layers-style nn.Sequential (model.py:25-45)."""
    out = []
    pool_names = {"conv1_2": "pool1_stage1", "conv2_2": "pool2_stage1", "conv3_4": "pool3_stage1"}
    for c in specs:
        out.append((c.name, nn.Conv2d(c.cin, c.cout, c.k, 1, c.k // 2)))
        if c.act == netspec.ACT_RELU:
            out.append(("relu_" + c.name, nn.ReLU(inplace=True)))
        elif c.act == netspec.ACT_PRELU:
            out.append((c.prelu, nn.PReLU(c.cout)))
        if c.name in pools_after:
            out.append((pool_names[c.name], nn.MaxPool2d(2, 2, 0)))
    return out


_POOLS = ("conv1_2", "conv2_2", "conv3_4")


class _NativeNet(nn.Module):
    KIND = None

    def __init__(self):
        super().__init__()
        object.__setattr__(self, "_native_net", None)
        object.__setattr__(self, "_native_key", None)

    def _param_key(self):
        """(storage, in-place version) of every parameter: load_state_dict / in-place edits bump
        the versions, a replaced parameter changes its storage.  The modules holding parameters
        are listed once (re-listed when a top-level child is replaced): walking
        self.parameters() per call cost ~0.3 ms per net on every per-frame call."""
        top = tuple(map(id, self._modules.values()))
        cache = self.__dict__.get("_native_mods")
        if cache is None or cache[0] != top:
            cache = (top, [m for m in self.modules() if m._parameters])
            object.__setattr__(self, "_native_mods", cache)
        return tuple((p.data_ptr(), p._version) for m in cache[1] for p in m._parameters.values() if p is not None)

    def _freeze(self):
        for p in self.parameters():       # model.py:167-168, 298-299, 391-392
            p.requires_grad = False

    def caffe_weights(self) -> dict:
        return {caffe_name(k): v for k, v in self.state_dict().items()}

    def native(self, device_index: int) -> rt.Net:
        """The libislpose net for this module on `device_index`, with current parameters."""
        net = self._native_net
        if net is None or net.device != device_index:
            net = rt.Net(self.KIND, device_index)
            object.__setattr__(self, "_native_net", net)
            object.__setattr__(self, "_native_key", None)
        key = self._param_key()
        if key != self._native_key:
            net.load_weights(self.caffe_weights())
            object.__setattr__(self, "_native_key", key)
        return net

    def forward(self, x):
        if not torch.cuda.is_available():
            if x.is_cuda:
                raise RuntimeError("a CUDA tensor without a visible HIP device")
            with torch.no_grad():
                return self.cpu_forward(x.float())
        dev = x.device if x.is_cuda else torch.device("cuda", torch.cuda.current_device())
        with torch.no_grad():
            out = self.native(dev.index if dev.index is not None else torch.cuda.current_device()).forward(
                x.to(dev, torch.float32).contiguous())
        if x.is_cuda:
            return out
        return tuple(o.cpu() for o in out) if isinstance(out, tuple) else out.cpu()


class bodypose_25_model(_NativeNet):
    """body_25 (model.py:66-207): forward(x) -> (PAF [N,52,h/8,w/8], heat [N,26,h/8,w/8])."""
    KIND = rt.ISL_BODY25

    def __init__(self):
        super().__init__()
        specs = netspec.body25_convs()
        self.model0 = nn.Sequential(OrderedDict(_conv_layers(specs[:12], _POOLS)))
        by_name = {c.name: c for c in specs}
        blocks = OrderedDict()
        tags = ["stage%d_L2" % s for s in range(4)] + ["stage0_L1", "stage1_L1"]
        for tag in tags:
            for b in range(1, 6):
                blocks["Mconv%d_%s" % (b, tag)] = [by_name["Mconv%d_%s_%d" % (b, tag, j)] for j in range(3)]
            blocks["Mconv6_7_%s" % tag] = [by_name["Mconv6_%s" % tag], by_name["Mconv7_%s" % tag]]
        # make_layers_Mconv: one nn.Sequential(conv[, PReLU]) per conv in a ModuleList (model.py:48-64)
        self.models = nn.ModuleDict(OrderedDict(
            (k, nn.ModuleList([nn.Sequential(OrderedDict(_conv_layers([c]))) for c in v])) for k, v in blocks.items()))
        self._freeze()

    def cpu_forward(self, x):
        """model.py:171-207: four L2 stages, then two L1 stages; each Mconv block concatenates
        its three convs' outputs."""
        def block(t, key):
            outs = []
            for m in self.models[key]:
                t = m(t)
                outs.append(t)
            return torch.cat(outs, 1)

        def stage(t, tag):
            for v in range(1, 6):
                t = block(t, "Mconv%d_%s" % (v, tag))
            m67 = self.models["Mconv6_7_%s" % tag]
            return m67[1](m67[0](t))

        out0 = self.model0(x)
        t = out0
        for s in range(4):
            l2 = stage(t, "stage%d_L2" % s)
            t = torch.cat([out0, l2], 1)
        l1 = stage(t, "stage0_L1")
        l1 = stage(torch.cat([out0, l1, l2], 1), "stage1_L1")
        return l2, l1


class bodypose_model(_NativeNet):
    """COCO-18 (model.py:210-329): forward(x) -> (PAF [N,38,..], heat [N,19,..])."""
    KIND = rt.ISL_COCO

    def __init__(self):
        super().__init__()
        specs = netspec.coco_convs()
        self.model0 = nn.Sequential(OrderedDict(_conv_layers(specs[:12], _POOLS)))
        rest = specs[12:]
        groups = OrderedDict()
        groups["model1_1"] = [c for c in rest if c.name.startswith("conv5_") and c.name.endswith("_L1")]
        groups["model1_2"] = [c for c in rest if c.name.startswith("conv5_") and c.name.endswith("_L2")]
        for i in range(2, 7):
            groups["model%d_1" % i] = [c for c in rest if ("_stage%d_L1" % i) in c.name]
            groups["model%d_2" % i] = [c for c in rest if ("_stage%d_L2" % i) in c.name]
        # registration order of model.py:285-297: model1_1 .. model6_1, then model1_2 .. model6_2
        for br in (1, 2):
            for i in range(1, 7):
                k = "model%d_%d" % (i, br)
                setattr(self, k, nn.Sequential(OrderedDict(_conv_layers(groups[k]))))
        self._freeze()

    def cpu_forward(self, x):
        """model.py:301-328: six two-branch stages over the VGG features."""
        out1 = self.model0(x)
        t = out1
        for i in range(1, 6):
            t = torch.cat([getattr(self, "model%d_1" % i)(t), getattr(self, "model%d_2" % i)(t), out1], 1)
        return self.model6_1(t), self.model6_2(t)


class handpose_model(_NativeNet):
    """hand (model.py:331-407): forward(x) -> heat [N,22,h/8,w/8]."""
    KIND = rt.ISL_HAND

    def __init__(self):
        super().__init__()
        specs = netspec.hand_convs()
        self.model1_0 = nn.Sequential(OrderedDict(_conv_layers(specs[:15], _POOLS)))
        self.model1_1 = nn.Sequential(OrderedDict(_conv_layers(specs[15:17])))
        for i in range(2, 7):
            setattr(self, "model%d" % i,
                    nn.Sequential(OrderedDict(_conv_layers([c for c in specs[17:] if c.name.endswith("_stage%d" % i)]))))
        self._freeze()

    def cpu_forward(self, x):
        """model.py:394-407: the CPM front, then five refinement stages."""
        out1_0 = self.model1_0(x)
        t = self.model1_1(out1_0)
        for i in range(2, 7):
            t = getattr(self, "model%d" % i)(torch.cat([t, out1_0], 1))
        return t
