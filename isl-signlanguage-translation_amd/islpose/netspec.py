"""Parameter tables of the three OpenPose networks.

Each network is described as the ordered list of its convolutions, with the
caffe parameter names the reference's weight files use (the flat
``{caffe_layer.weight|bias: FloatTensor}`` dict that ``util.transfer``
consumes, /root/reference/src/util.py:35-44) and the activation that follows
each convolution.

This table only names parameters and their shapes (for loading / synthesising
weight dicts on the host).  The device-side graph (buffer plan, concat slices,
launch order) is built natively by ``csrc/graph.cpp``.

Reference: /root/reference/src/model.py
  * body_25  ``bodypose_25_model``  model.py:66-207
  * COCO-18  ``bodypose_model``     model.py:210-329
  * hand     ``handpose_model``     model.py:331-407
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

ACT_NONE, ACT_RELU, ACT_PRELU = 0, 1, 2

KIND_BODY25, KIND_COCO, KIND_HAND = 0, 1, 2
KIND_NAMES = {KIND_BODY25: "body25", KIND_COCO: "coco", KIND_HAND: "hand"}


@dataclass(frozen=True)
class ConvSpec:
    name: str            # caffe layer name, e.g. "Mconv1_stage0_L2_0"
    cin: int
    cout: int
    k: int
    act: int             # ACT_*
    prelu: Optional[str]  # caffe name of the PReLU slope tensor, if act == ACT_PRELU

    @property
    def params(self):
        out = [(self.name + ".weight", (self.cout, self.cin, self.k, self.k)),
               (self.name + ".bias", (self.cout,))]
        if self.prelu is not None:
            out.append((self.prelu + ".weight", (self.cout,)))
        return out


def _vgg_front(prelu_layers=(), extended_hand=False):
    # model.py:75-91 (body_25), :220-236 (COCO), :339-358 (hand)
    layers = [("conv1_1", 3, 64), ("conv1_2", 64, 64), ("pool",),
              ("conv2_1", 64, 128), ("conv2_2", 128, 128), ("pool",),
              ("conv3_1", 128, 256), ("conv3_2", 256, 256), ("conv3_3", 256, 256),
              ("conv3_4", 256, 256), ("pool",),
              ("conv4_1", 256, 512), ("conv4_2", 512, 512)]
    if extended_hand:
        layers += [("conv4_3", 512, 512), ("conv4_4", 512, 512), ("conv5_1", 512, 512),
                   ("conv5_2", 512, 512), ("conv5_3_CPM", 512, 128)]
    else:
        layers += [("conv4_3_CPM", 512, 256), ("conv4_4_CPM", 256, 128)]
    out = []
    for l in layers:
        if l[0] == "pool":
            continue
        name, cin, cout = l
        if name in prelu_layers:
            # make_layers names the PReLU 'prelu' + name[4:]  (model.py:43)
            out.append(ConvSpec(name, cin, cout, 3, ACT_PRELU, "prelu" + name[4:]))
        else:
            out.append(ConvSpec(name, cin, cout, 3, ACT_RELU, None))
    return out


def body25_convs() -> List[ConvSpec]:
    """bodypose_25_model, model.py:66-165 (114 convolutions)."""
    convs = _vgg_front(prelu_layers=("conv4_2", "conv4_3_CPM", "conv4_4_CPM"))
    no_act = {"Mconv7_stage0_L1", "Mconv7_stage0_L2", "Mconv7_stage1_L1", "Mconv7_stage1_L2",
              "Mconv7_stage2_L2", "Mconv7_stage3_L2"}  # model.py:70-72

    def mconv(name, cin, cout, k):
        if name in no_act:
            return ConvSpec(name, cin, cout, k, ACT_NONE, None)
        # make_layers_Mconv: every non-final Mconv gets PReLU 'Mprelu'+name[5:]  (model.py:61-62)
        return ConvSpec(name, cin, cout, k, ACT_PRELU, "Mprelu" + name[5:])

    def stage(tag, cin, width, c6, cout):
        out = []
        for b in range(1, 6):
            c_in_block = cin if b == 1 else 3 * width
            for j in range(3):
                out.append(mconv("Mconv%d_%s_%d" % (b, tag, j), c_in_block if j == 0 else width, width, 3))
        out.append(mconv("Mconv6_%s" % tag, 3 * width, c6, 1))
        out.append(mconv("Mconv7_%s" % tag, c6, cout, 1))
        return out

    convs += stage("stage0_L2", 128, 96, 256, 52)          # model.py:96-110
    for s in range(1, 4):                                  # model.py:112-127
        convs += stage("stage%d_L2" % s, 180, 128, 512, 52)
    convs += stage("stage0_L1", 180, 96, 256, 26)          # model.py:131-145
    convs += stage("stage1_L1", 206, 128, 512, 26)         # model.py:147-161
    return convs


def coco_convs() -> List[ConvSpec]:
    """bodypose_model, model.py:210-299."""
    # model.py:215-218: note 'Mconv7_stage6_L1' appears twice and
    # 'Mconv7_stage6_L2' is missing -> the final heat conv keeps its ReLU.
    no_relu = {"conv5_5_CPM_L1", "conv5_5_CPM_L2", "Mconv7_stage2_L1", "Mconv7_stage2_L2",
               "Mconv7_stage3_L1", "Mconv7_stage3_L2", "Mconv7_stage4_L1", "Mconv7_stage4_L2",
               "Mconv7_stage5_L1", "Mconv7_stage5_L2", "Mconv7_stage6_L1"}

    def c(name, cin, cout, k):
        return ConvSpec(name, cin, cout, k, ACT_NONE if name in no_relu else ACT_RELU, None)

    convs = _vgg_front()
    for br, cout in ((1, 38), (2, 19)):                     # model.py:240-254
        convs += [c("conv5_1_CPM_L%d" % br, 128, 128, 3), c("conv5_2_CPM_L%d" % br, 128, 128, 3),
                  c("conv5_3_CPM_L%d" % br, 128, 128, 3), c("conv5_4_CPM_L%d" % br, 128, 512, 1),
                  c("conv5_5_CPM_L%d" % br, 512, cout, 1)]
    for i in range(2, 7):                                   # model.py:261-280
        for br, cout in ((1, 38), (2, 19)):
            convs += [c("Mconv1_stage%d_L%d" % (i, br), 185, 128, 7)]
            convs += [c("Mconv%d_stage%d_L%d" % (j, i, br), 128, 128, 7) for j in range(2, 6)]
            convs += [c("Mconv6_stage%d_L%d" % (i, br), 128, 128, 1),
                      c("Mconv7_stage%d_L%d" % (i, br), 128, cout, 1)]
    return convs


def hand_convs() -> List[ConvSpec]:
    """handpose_model, model.py:331-392."""
    no_relu = {"conv6_2_CPM", "Mconv7_stage2", "Mconv7_stage3", "Mconv7_stage4",
               "Mconv7_stage5", "Mconv7_stage6"}               # model.py:336-337

    def c(name, cin, cout, k):
        return ConvSpec(name, cin, cout, k, ACT_NONE if name in no_relu else ACT_RELU, None)

    convs = _vgg_front(extended_hand=True)
    convs += [c("conv6_1_CPM", 128, 512, 1), c("conv6_2_CPM", 512, 22, 1)]
    for i in range(2, 7):
        convs += [c("Mconv1_stage%d" % i, 150, 128, 7)]
        convs += [c("Mconv%d_stage%d" % (j, i), 128, 128, 7) for j in range(2, 6)]
        convs += [c("Mconv6_stage%d" % i, 128, 128, 1), c("Mconv7_stage%d" % i, 128, 22, 1)]
    return convs


def convs_for(kind: int) -> List[ConvSpec]:
    return {KIND_BODY25: body25_convs, KIND_COCO: coco_convs, KIND_HAND: hand_convs}[kind]()


def param_shapes(kind: int):
    """Ordered list of (caffe_name, shape) for every parameter of the network."""
    out = []
    for c in convs_for(kind):
        out += c.params
    return out


def conv_flops(kind: int, h: int, w: int) -> int:
    """Algorithmic conv FLOPs (2*Cout*Cin*k*k*Ho*Wo summed) for one frame at net input h x w."""
    total = 0
    hh, ww = h, w
    pools_after = {"conv1_2", "conv2_2", "conv3_4"}
    for c in convs_for(kind):
        total += 2 * c.cout * c.cin * c.k * c.k * hh * ww
        if c.name in pools_after:
            hh, ww = hh // 2, ww // 2
    return total
