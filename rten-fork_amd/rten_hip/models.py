"""Synthetic model definitions for the benchmark configs (BASELINE.json).

No checkpoints or network exist here, so models are built with seeded
random weights of the real architectures, in the operator mix RTen receives
from an ONNX export with BatchNorm folded into Conv (tools/export-timm-model.py
exports with torch.onnx constant folding):

- ResNet-50 v1.5 (timm/torchvision ``resnet50``): Conv(+bias) / Relu / MaxPool
  / Add / GlobalAveragePool / Flatten / Gemm.  He-uniform weights
  U(+-sqrt(6/fan_in)), biases U(+-0.01), the last conv of every bottleneck
  scaled by 0.2 so activations stay O(1) through 16 residual blocks
  (SURVEY.md §8d).
- MobileNetV2 (width 1.0): Conv / depthwise Conv / Clip(0, 6) / Add /
  GlobalAveragePool / Flatten / Gemm.
"""
from __future__ import annotations

import numpy as np

from .graph import ModelSpec

RESNET50_GFLOP_PER_IMAGE = 8.178  # 2*MACs over 53 convs + FC
MOBILENETV2_GFLOP_PER_IMAGE = 0.6015


class _Init:
    def __init__(self, seed: int):
        self.rng = np.random.default_rng(seed)

    def conv(self, cout, cin, kh, kw, scale=1.0):
        fan_in = cin * kh * kw
        lim = np.sqrt(6.0 / fan_in) * scale
        w = self.rng.uniform(-lim, lim, size=(cout, cin, kh, kw)).astype(np.float32)
        b = self.rng.uniform(-0.01, 0.01, size=(cout,)).astype(np.float32)
        return w, b

    def fc(self, cout, cin):
        lim = np.sqrt(6.0 / cin)
        w = self.rng.uniform(-lim, lim, size=(cout, cin)).astype(np.float32)
        b = self.rng.uniform(-0.01, 0.01, size=(cout,)).astype(np.float32)
        return w, b


def _conv(m: ModelSpec, init: _Init, name, x, cin, cout, k, stride=1, pad=0, groups=1,
          scale=1.0, bn=False):
    w, b = init.conv(cout, cin // groups, k, k, scale)
    wn = m.const(f"{name}.weight", w)
    attrs = {"pads": [pad] * 4, "strides": [stride, stride], "dilations": [1, 1], "groups": groups}
    if not bn:
        return m.op("Conv", [x, wn, m.const(f"{name}.bias", b)], attrs, name=name)
    # An export without BN folding (torchvision layout: bias-free conv, then
    # BatchNormalization with its running statistics).
    y = m.op("Conv", [x, wn], attrs, name=name)
    rng = init.rng
    p = [rng.uniform(0.8, 1.2, cout), rng.uniform(-0.1, 0.1, cout), rng.uniform(-0.1, 0.1, cout),
         rng.uniform(0.5, 1.5, cout)]
    scale_n, bias_n, mean_n, var_n = (m.const(f"{name}.bn.{k}", v.astype(np.float32))
                                      for k, v in zip(("weight", "bias", "running_mean", "running_var"), p))
    return m.op("BatchNormalization", [y, scale_n, bias_n, mean_n, var_n], {"epsilon": 1e-5}, name=f"{name}.bn")


def resnet50(num_classes: int = 1000, seed: int = 4321, unfolded_bn: bool = False) -> ModelSpec:
    """ResNet-50 v1.5 (stride on the 3x3 conv), NCHW input [N,3,224,224]; BN
    folded into the convs (the benchmark export), or with ``unfolded_bn`` every
    conv bias-free and followed by a BatchNormalization node."""
    m = ModelSpec("resnet50_bn" if unfolded_bn else "resnet50")
    init = _Init(seed)
    x = m.value("input")
    m.inputs = ["input"]
    bn = unfolded_bn
    h = _conv(m, init, "conv1", x, 3, 64, 7, stride=2, pad=3, bn=bn)
    h = m.op("Relu", [h], name="relu1")
    h = m.op("MaxPool", [h], {"kernel_size": [3, 3], "strides": [2, 2], "pads": [1, 1, 1, 1]},
             name="maxpool")
    cin = 64
    for li, (width, blocks, stride) in enumerate([(64, 3, 1), (128, 4, 2), (256, 6, 2),
                                                  (512, 3, 2)]):
        for bi in range(blocks):
            s = stride if bi == 0 else 1
            pre = f"layer{li + 1}.{bi}"
            cout = width * 4
            t = _conv(m, init, f"{pre}.conv1", h, cin, width, 1, bn=bn)
            t = m.op("Relu", [t], name=f"{pre}.relu1")
            t = _conv(m, init, f"{pre}.conv2", t, width, width, 3, stride=s, pad=1, bn=bn)
            t = m.op("Relu", [t], name=f"{pre}.relu2")
            t = _conv(m, init, f"{pre}.conv3", t, width, cout, 1, scale=0.2, bn=bn)
            if bi == 0:
                ident = _conv(m, init, f"{pre}.downsample", h, cin, cout, 1, stride=s, bn=bn)
            else:
                ident = h
            t = m.op("Add", [t, ident], name=f"{pre}.add")
            h = m.op("Relu", [t], name=f"{pre}.relu3")
            cin = cout
    h = m.op("GlobalAveragePool", [h], name="avgpool")
    h = m.op("Flatten", [h], {"axis": 1}, name="flatten")
    w, b = init.fc(num_classes, 2048)
    h = m.op("Gemm", [h, m.const("fc.weight", w), m.const("fc.bias", b)],
             {"alpha": 1.0, "beta": 1.0, "transA": 0, "transB": 1}, name="fc")
    m.outputs = [h]
    return m


def mobilenet_v2(num_classes: int = 1000, seed: int = 4321) -> ModelSpec:
    """MobileNetV2 1.0 (torchvision layout), BN folded, ReLU6 = Clip(0, 6)."""
    m = ModelSpec("mobilenet_v2")
    init = _Init(seed)
    x = m.value("input")
    m.inputs = ["input"]
    zero = m.const("clip.min", np.array(0.0, np.float32))
    six = m.const("clip.max", np.array(6.0, np.float32))

    def relu6(t, name):
        return m.op("Clip", [t, zero, six], name=name)

    h = relu6(_conv(m, init, "features.0", x, 3, 32, 3, stride=2, pad=1), "features.0.relu6")
    cin = 32
    cfg = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1),
           (6, 160, 3, 2), (6, 320, 1, 1)]
    idx = 1
    for t_exp, c, n, s in cfg:
        for i in range(n):
            stride = s if i == 0 else 1
            pre = f"features.{idx}"
            hidden = cin * t_exp
            y = h
            if t_exp != 1:
                y = relu6(_conv(m, init, f"{pre}.expand", y, cin, hidden, 1), f"{pre}.expand.relu6")
            y = relu6(_conv(m, init, f"{pre}.dw", y, hidden, hidden, 3, stride=stride, pad=1,
                            groups=hidden), f"{pre}.dw.relu6")
            y = _conv(m, init, f"{pre}.project", y, hidden, c, 1, scale=0.5)
            if stride == 1 and cin == c:
                y = m.op("Add", [y, h], name=f"{pre}.add")
            h = y
            cin = c
            idx += 1
    h = relu6(_conv(m, init, "features.18", h, 320, 1280, 1), "features.18.relu6")
    h = m.op("GlobalAveragePool", [h], name="avgpool")
    h = m.op("Flatten", [h], {"axis": 1}, name="flatten")
    w, b = init.fc(num_classes, 1280)
    h = m.op("Gemm", [h, m.const("classifier.weight", w), m.const("classifier.bias", b)],
             {"alpha": 1.0, "beta": 1.0, "transA": 0, "transB": 1}, name="classifier")
    m.outputs = [h]
    return m


def conv_flops(spec: ModelSpec, batch: int, hw: int = 224) -> float:
    """2*MAC count of every Conv and Gemm in ``spec`` at input [batch,3,hw,hw]
    (used for the roofline figure; cross-checked against SURVEY.md App. A)."""
    shapes = {spec.inputs[0]: (batch, 3, hw, hw)}
    consts = {n.name: n.data.shape for n in spec.nodes if n.kind == "const"}
    total = 0.0
    for n in spec.nodes:
        if n.kind != "op":
            continue
        xs = shapes.get(n.inputs[0]) if n.inputs and n.inputs[0] in shapes else None
        if n.op_type == "Conv":
            o, ci, kh, kw = consts[n.inputs[1]]
            N, C, H, W = xs
            p, s = n.attrs["pads"], n.attrs["strides"]
            oh = (H + p[0] + p[2] - kh) // s[0] + 1
            ow = (W + p[1] + p[3] - kw) // s[1] + 1
            total += 2.0 * N * o * oh * ow * ci * kh * kw
            shapes[n.outputs[0]] = (N, o, oh, ow)
        elif n.op_type == "MaxPool":
            N, C, H, W = xs
            k, s, p = n.attrs["kernel_size"], n.attrs["strides"], n.attrs["pads"]
            shapes[n.outputs[0]] = (N, C, (H + p[0] + p[2] - k[0]) // s[0] + 1,
                                    (W + p[1] + p[3] - k[1]) // s[1] + 1)
            total += 4.0 * (N * C * H * W + float(np.prod(shapes[n.outputs[0]])))  # read + write
        elif n.op_type == "GlobalAveragePool":
            shapes[n.outputs[0]] = (xs[0], xs[1], 1, 1)
        elif n.op_type == "Flatten":
            shapes[n.outputs[0]] = (xs[0], int(np.prod(xs[1:])))
        elif n.op_type == "Gemm":
            o, k = consts[n.inputs[1]]
            total += 2.0 * xs[0] * o * k
            shapes[n.outputs[0]] = (xs[0], o)
        else:
            shapes[n.outputs[0]] = xs
    return total


def _expand_dw_fused(cin: int, h: int, w: int, stride: int = 1) -> bool:
    """Whether csrc/mbconv.hip runs an expand -> depthwise pair of these
    shapes as one kernel by default (expand_dw_eligible's default policy: the
    banded kernel for C_in 16 / 24, and 32 at stride 2).  Kept in step with
    the executor by tests/test_conv_pointwise_gpu.py (fused pairs counted in
    the timing report)."""
    banded = w % 4 == 0 and w // 4 <= 256 // 3
    return banded and (cin in (16, 24) or (cin == 32 and stride == 2))


def _dw_project_fused(c: int, h: int, w: int, m: int, stride: int) -> bool:
    """Whether csrc/dw_project.hip runs a depthwise 3x3 -> 1x1 projection pair
    of these shapes as one kernel (dw_project_eligible; pads 1 checked by the
    caller through the output size)."""
    return c == 32 and w == 112 and m <= 32 and stride == 1


def _stem_dw_project_fused(stem, xshape, consts) -> bool:
    """Whether csrc/dw_project.hip also runs the stem conv feeding a fused
    depthwise -> projection pair (stem_dw_project_eligible: 3 -> 32 channels,
    3x3 / 2, pads 1 at the top and left, 224 input columns)."""
    o, ci, kh, kw = consts[stem.inputs[1]]
    p, s = stem.attrs["pads"], stem.attrs["strides"]
    return (ci == 3 and (kh, kw) == (3, 3) and list(s) == [2, 2] and p[0] == 1 and p[1] == 1 and o == 32 and
            stem.attrs.get("groups", 1) == 1 and xshape[1] == 3 and xshape[3] == 224 and
            (xshape[3] + p[1] + p[3] - 3) // 2 + 1 == 112)


def expand_dw_pairs(spec: ModelSpec, batch: int = 1, hw: int = 224) -> int:
    """Expand -> depthwise pairs of ``spec`` the executor fuses by default."""
    return int(conv_io_bytes(spec, batch, hw, count_pairs=True))


def _expand_dw_fusable(cin: int, h: int, w: int) -> bool:
    """Every pair a fused kernel can take (RTENHIP_EXPAND_DW=all)."""
    banded = cin in (16, 24, 32) and w % 4 == 0
    p = h * w
    g = (4 * 8) if p <= 64 else 16
    flat = p <= 256 and (cin * p + g * (p + 8)) * 4 <= 100 * 1024
    return banded or flat


def conv_io_bytes(spec: ModelSpec, batch: int, hw: int = 224, count_pairs: bool = False) -> float:
    """Algorithmic HBM bytes of every Conv (and the classifier Gemm) in
    ``spec`` at input [batch, 3, hw, hw], as the fused graph moves them: each
    conv reads its input and weights (+ bias) once and writes its output once;
    a residual Add fused into the conv's epilogue reads its other operand once;
    Relu / Clip ride in the epilogue (no traffic); an expand -> depthwise pair
    run as one kernel (mbconv.hip) neither writes nor reads the expand output,
    nor a depthwise -> projection pair (dw_project.hip) the depthwise output,
    nor MobileNetV2's stem fused into that pair the stem output.
    The HBM-roofline figure for bandwidth-bound models (MobileNetV2,
    SURVEY.md §8d)."""
    shapes = {spec.inputs[0]: (batch, 3, hw, hw)}
    consts = {n.name: n.data.shape for n in spec.nodes if n.kind == "const"}
    producer = {o: n for n in spec.nodes if n.kind == "op" for o in n.outputs}

    def source_conv(v, k=(1, 1)):
        """The k[0] x k[1] Conv behind value v (through a Clip / Relu), or None."""
        n = producer.get(v)
        if n is not None and n.op_type in ("Clip", "Relu"):
            n = producer.get(n.inputs[0])
        if n is None or n.op_type != "Conv" or consts[n.inputs[1]][2:] != k:
            return None
        return n

    expand_fused_dw = set()  # depthwise convs run with their expand conv

    fused_e, fused_d = set(), set()
    total = 0.0
    pairs = 0
    for n in spec.nodes:
        if n.kind != "op":
            continue
        xs = shapes.get(n.inputs[0]) if n.inputs and n.inputs[0] in shapes else None
        if n.op_type == "Conv":
            o, ci, kh, kw = consts[n.inputs[1]]
            N, C, H, W = xs
            p, s = n.attrs["pads"], n.attrs["strides"]
            oh = (H + p[0] + p[2] - kh) // s[0] + 1
            ow = (W + p[1] + p[3] - kw) // s[1] + 1
            rd, wr = N * C * H * W, N * o * oh * ow
            e = source_conv(n.inputs[0])
            if n.attrs.get("groups", 1) == C and (kh, kw) == (3, 3) and e is not None:
                ex = shapes[e.inputs[0]]
                if _expand_dw_fused(ex[1], ex[2], ex[3], s[0]):
                    pairs += 1
                    expand_fused_dw.add(n.name)
                    rd = 0  # the expand output never reaches HBM
                    total -= 4.0 * N * C * H * W  # nor is written by the expand
            d = source_conv(n.inputs[0], (3, 3)) if (kh, kw) == (1, 1) and n.attrs.get("groups", 1) == 1 else None
            if d is not None and d.name not in expand_fused_dw and d.attrs.get("groups", 1) == C:
                dx = shapes[d.inputs[0]]
                if dx[2:] == (H, W) and _dw_project_fused(C, H, W, o, d.attrs["strides"][0]):
                    rd = 0  # the depthwise output never reaches HBM
                    total -= 4.0 * N * C * H * W  # nor is written by the depthwise conv
                    st = source_conv(d.inputs[0], (3, 3))
                    if st is not None and _stem_dw_project_fused(st, shapes[st.inputs[0]], consts):
                        total -= 2 * 4.0 * float(np.prod(dx))  # the stem output: neither written nor read
            total += 4.0 * (rd + wr + o * ci * kh * kw + o)
            shapes[n.outputs[0]] = (N, o, oh, ow)
        elif n.op_type == "Add":
            total += 4.0 * float(np.prod(xs))  # the residual operand
            shapes[n.outputs[0]] = xs
        elif n.op_type == "MaxPool":
            N, C, H, W = xs
            k, s, p = n.attrs["kernel_size"], n.attrs["strides"], n.attrs["pads"]
            shapes[n.outputs[0]] = (N, C, (H + p[0] + p[2] - k[0]) // s[0] + 1,
                                    (W + p[1] + p[3] - k[1]) // s[1] + 1)
            total += 4.0 * (N * C * H * W + float(np.prod(shapes[n.outputs[0]])))  # read + write
        elif n.op_type == "GlobalAveragePool":
            shapes[n.outputs[0]] = (xs[0], xs[1], 1, 1)
        elif n.op_type == "Flatten":
            shapes[n.outputs[0]] = (xs[0], int(np.prod(xs[1:])))
        elif n.op_type == "Gemm":
            o, k = consts[n.inputs[1]]
            total += 4.0 * (xs[0] * k + o * k + o + xs[0] * o)
            shapes[n.outputs[0]] = (xs[0], o)
        else:
            shapes[n.outputs[0]] = xs
    return pairs if count_pairs else total


BERT_BASE_GFLOP_PER_SEQ128 = 22.347  # SURVEY.md App. A.3 (encoder, seq 128)


def bert_encoder(layers: int = 12, hidden: int = 768, heads: int = 12, ffn: int = 3072,
                 seq: int = 128, eps: float = 1e-12, seed: int = 4321, embeddings: bool = False,
                 vocab: int = 30522, max_pos: int = 512, type_vocab: int = 2,
                 mask_op: str = "mul", unfused: bool = False) -> ModelSpec:
    """BERT-base encoder stack in the operator mix of an ONNX export as RTen
    runs it after its own fusions (GELU and LayerNormalization fused,
    src/optimize.rs): per layer Q/K/V MatMul+Add, Reshape/Transpose to heads,
    QK^T MatMul, Div by sqrt(d_head), Add of the additive attention mask,
    Softmax, AV MatMul, Transpose/Reshape back, output MatMul+Add, residual
    Add + LayerNormalization, FFN MatMul+Add -> Gelu -> MatMul+Add, residual
    Add + LayerNormalization.

    Inputs: ``hidden_states`` [B, S, hidden] (the embedding output: the token
    Gather is outside the f32 hot path) and ``attention_mask`` [B, 1, 1, S]
    (additive; zeros for the all-ones mask rten-cli uses, rten-cli main.rs).
    Weights U(+-0.05) (BERT's N(0, 0.02) init has the same scale), biases
    U(+-0.01), LayerNorm gamma ~1, beta ~0.

    ``embeddings=True`` prepends the embedding and mask subgraph of the ONNX
    export (int32 inputs ``input_ids``, ``token_type_ids``, ``attention_mask``
    [B, S]): word / position / token-type Gathers, their sum and
    LayerNormalization; the 0/1 mask becomes the additive one through
    Unsqueeze x2 -> Cast(Float) -> Sub(1, .) -> Mul(-10000) (``mask_op="mul"``,
    the classic export) or Where(mask, 0, -10000) (``mask_op="where"``).

    ``unfused=True`` emits the graph as an ONNX export hands it to RTen,
    before RTen's optimizer (src/optimize.rs:286-518) runs: LayerNorm as
    ReduceMean(-1) / Sub / Pow(2) / ReduceMean(-1) / Add(eps) / Sqrt / Div /
    Mul(gamma) / Add(beta), GELU as nn.GELU's Div(sqrt 2) / Erf / Add(1) / Mul /
    Mul(0.5), the head split and merge reshapes through a Shape -> Gather ->
    Unsqueeze -> Concat shape subgraph, the position ids as a Slice of a
    [1, max_pos] buffer up to the input's sequence length, and the attention
    scale as Sqrt of a constant (folded by constant propagation).  After the
    optimizer it is the fused graph, weights and bits included."""
    m = ModelSpec(("bert_base" if layers == 12 else f"bert_l{layers}") + ("_emb" if embeddings else "") +
                  ("_onnx" if unfused else ""))
    rng = np.random.default_rng(seed)
    dh = hidden // heads
    if embeddings:
        ids, types, am = m.value("input_ids"), m.value("token_type_ids"), m.value("attention_mask")
        m.inputs = ["input_ids", "token_type_ids", "attention_mask"]
        wte = m.const("emb.word", rng.uniform(-0.05, 0.05, (vocab, hidden)).astype(np.float32))
        wpe = m.const("emb.position", rng.uniform(-0.05, 0.05, (max_pos, hidden)).astype(np.float32))
        wtt = m.const("emb.token_type", rng.uniform(-0.05, 0.05, (type_vocab, hidden)).astype(np.float32))
        if unfused:
            # position_ids[:, :seq_len] of the registered [1, max_pos] buffer
            buf = m.const("emb.position_ids", np.arange(max_pos, dtype=np.int32).reshape(1, max_pos))
            ishape = m.op("Shape", [ids], name="emb.ids.shape")
            slen = m.op("Gather", [ishape, m.const("emb.idx1", np.array(1, np.int32))], {"axis": 0},
                        name="emb.seq_len")
            slen = m.op("Unsqueeze", [slen, m.const("emb.axes0", np.array([0], np.int32))],
                        name="emb.seq_len.unsqueeze")
            pos_ids = m.op("Slice", [buf, m.const("emb.start0", np.array([0], np.int32)), slen,
                                     m.const("emb.axes1", np.array([1], np.int32))], name="emb.position_ids.slice")
        else:
            pos_ids = m.const("emb.position_ids", np.arange(seq, dtype=np.int32).reshape(1, seq))
        e = m.op("Gather", [wte, ids], {"axis": 0}, name="emb.word.gather")
        e = m.op("Add", [e, m.op("Gather", [wtt, types], {"axis": 0}, name="emb.type.gather")],
                 name="emb.add_type")
        e = m.op("Add", [e, m.op("Gather", [wpe, pos_ids], {"axis": 0}, name="emb.pos.gather")],
                 name="emb.add_pos")
        g0 = m.const("emb.ln.gamma", (1.0 + rng.uniform(-0.1, 0.1, (hidden,))).astype(np.float32))
        b0 = m.const("emb.ln.beta", rng.uniform(-0.1, 0.1, (hidden,)).astype(np.float32))
        x = _layer_norm(m, "emb.ln", e, g0, b0, eps, unfused)
        ax1 = m.const("mask.axes1", np.array([1], np.int32))
        ax2 = m.const("mask.axes2", np.array([2], np.int32))
        mk = m.op("Unsqueeze", [am, ax1], name="mask.unsqueeze1")
        mk = m.op("Unsqueeze", [mk, ax2], name="mask.unsqueeze2")
        if mask_op == "where":
            zero = m.const("mask.zero", np.array([0.0], np.float32))
            neg = m.const("mask.neg", np.array([-10000.0], np.float32))
            mask = m.op("Where", [mk, zero, neg], name="mask.where")
        else:
            mf = m.op("Cast", [mk], {"to": 1}, name="mask.cast")
            one = m.const("mask.one", np.array([1.0], np.float32))
            neg = m.const("mask.neg", np.array([-10000.0], np.float32))
            mask = m.op("Mul", [m.op("Sub", [one, mf], name="mask.invert"), neg], name="mask.scale")
    else:
        x = m.value("hidden_states")
        mask = m.value("attention_mask")
        m.inputs = ["hidden_states", "attention_mask"]

    def lin(name, h, cin, cout):
        w = m.const(f"{name}.weight", rng.uniform(-0.05, 0.05, (cin, cout)).astype(np.float32))
        b = m.const(f"{name}.bias", rng.uniform(-0.01, 0.01, (cout,)).astype(np.float32))
        y = m.op("MatMul", [h, w], name=f"{name}.matmul")
        return m.op("Add", [y, b], name=f"{name}.add")

    def ln(name, h):
        g = m.const(f"{name}.gamma", (1.0 + rng.uniform(-0.1, 0.1, (hidden,))).astype(np.float32))
        b = m.const(f"{name}.beta", rng.uniform(-0.1, 0.1, (hidden,)).astype(np.float32))
        return _layer_norm(m, name, h, g, b, eps, unfused)

    if unfused:
        # scale = Sqrt(d_head) computed in the graph (constant propagation folds it)
        scale = m.op("Sqrt", [m.const("attn.d_head", np.array(float(dh), np.float32))], name="attn.scale")
        c_heads = m.const("shape.heads_dh", np.array([heads, dh], np.int32))
        c_hidden = m.const("shape.hidden", np.array([hidden], np.int32))
        idx0 = m.const("shape.idx0", np.array(0, np.int32))
        idx1 = m.const("shape.idx1", np.array(1, np.int32))
        ax0 = m.const("shape.axes0", np.array([0], np.int32))

        def dyn_shape(name, t, tail):
            # torch's x.size()[:2] + tail as ONNX exports it
            sh = m.op("Shape", [t], name=f"{name}.shape")
            d0 = m.op("Unsqueeze", [m.op("Gather", [sh, idx0], {"axis": 0}, name=f"{name}.d0"), ax0],
                      name=f"{name}.d0u")
            d1 = m.op("Unsqueeze", [m.op("Gather", [sh, idx1], {"axis": 0}, name=f"{name}.d1"), ax0],
                      name=f"{name}.d1u")
            return m.op("Concat", [d0, d1, tail], {"axis": 0}, name=f"{name}.concat")
    else:
        shape_heads = m.const("shape.heads", np.array([0, 0, heads, dh], np.float32))
        shape_merge = m.const("shape.merge", np.array([0, 0, hidden], np.float32))
        scale = m.const("attn.scale", np.array([np.sqrt(dh)], np.float32))
    h = x
    for i in range(layers):
        p = f"layer{i}"
        q = lin(f"{p}.q", h, hidden, hidden)
        k = lin(f"{p}.k", h, hidden, hidden)
        v = lin(f"{p}.v", h, hidden, hidden)
        if unfused:
            shape_heads = dyn_shape(f"{p}.heads", q, c_heads)
        q = m.op("Reshape", [q, shape_heads], name=f"{p}.q.reshape")
        q = m.op("Transpose", [q], {"perm": [0, 2, 1, 3]}, name=f"{p}.q.transpose")
        k = m.op("Reshape", [k, shape_heads], name=f"{p}.k.reshape")
        k = m.op("Transpose", [k], {"perm": [0, 2, 3, 1]}, name=f"{p}.k.transpose")
        v = m.op("Reshape", [v, shape_heads], name=f"{p}.v.reshape")
        v = m.op("Transpose", [v], {"perm": [0, 2, 1, 3]}, name=f"{p}.v.transpose")
        s = m.op("MatMul", [q, k], name=f"{p}.qk")
        s = m.op("Div", [s, scale], name=f"{p}.scale")
        s = m.op("Add", [s, mask], name=f"{p}.mask")
        s = m.op("Softmax", [s], {"axis": -1}, name=f"{p}.softmax")
        c = m.op("MatMul", [s, v], name=f"{p}.av")
        c = m.op("Transpose", [c], {"perm": [0, 2, 1, 3]}, name=f"{p}.ctx.transpose")
        if unfused:
            shape_merge = dyn_shape(f"{p}.merge", c, c_hidden)
        c = m.op("Reshape", [c, shape_merge], name=f"{p}.ctx.reshape")
        a = lin(f"{p}.attn_out", c, hidden, hidden)
        h1 = ln(f"{p}.ln1", m.op("Add", [a, h], name=f"{p}.res1"))
        f = lin(f"{p}.ffn1", h1, hidden, ffn)
        f = _gelu(m, f"{p}.gelu", f, unfused)
        f = lin(f"{p}.ffn2", f, ffn, hidden)
        h = ln(f"{p}.ln2", m.op("Add", [f, h1], name=f"{p}.res2"))
    m.outputs = [h]
    return m


def _layer_norm(m: ModelSpec, name, x, gamma, beta, eps, unfused):
    """LayerNormalization, or torch.onnx's decomposition of it (opset < 17)."""
    if not unfused:
        return m.op("LayerNormalization", [x, gamma, beta], {"axis": -1, "epsilon": eps}, name=name)
    mean = m.op("ReduceMean", [x], {"axes": [-1], "keep_dims": 1}, name=f"{name}.mean")
    d = m.op("Sub", [x, mean], name=f"{name}.sub")
    var = m.op("ReduceMean", [m.op("Pow", [d, m.const(f"{name}.two", np.array(2.0, np.float32))],
                                   name=f"{name}.pow")], {"axes": [-1], "keep_dims": 1}, name=f"{name}.var")
    den = m.op("Sqrt", [m.op("Add", [var, m.const(f"{name}.eps", np.array(eps, np.float32))],
                             name=f"{name}.add_eps")], name=f"{name}.sqrt")
    y = m.op("Div", [d, den], name=f"{name}.div")
    return m.op("Add", [m.op("Mul", [y, gamma], name=f"{name}.mul"), beta], name=name)


def _gelu(m: ModelSpec, name, x, unfused):
    """Gelu, or nn.GELU as ONNX exports it: x * (erf(x / sqrt 2) + 1) * 0.5."""
    if not unfused:
        return m.op("Gelu", [x], name=name)
    e = m.op("Erf", [m.op("Div", [x, m.const(f"{name}.sqrt2", np.array(np.sqrt(2.0), np.float32))],
                          name=f"{name}.div")], name=f"{name}.erf")
    a = m.op("Add", [e, m.const(f"{name}.one", np.array(1.0, np.float32))], name=f"{name}.add")
    return m.op("Mul", [m.op("Mul", [x, a], name=f"{name}.mul"),
                        m.const(f"{name}.half", np.array(0.5, np.float32))], name=name)


def bert_flops(layers: int = 12, hidden: int = 768, heads: int = 12, ffn: int = 3072,
               seq: int = 128) -> float:
    """2*MACs per sequence of the encoder's MatMuls."""
    proj = 4 * seq * hidden * hidden + 2 * seq * hidden * ffn
    attn = 2 * seq * seq * hidden
    return 2.0 * layers * (proj + attn)
