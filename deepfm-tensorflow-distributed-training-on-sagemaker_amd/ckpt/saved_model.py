"""Hand-encoded TF1 ``saved_model.pb`` (reference C33 / SURVEY §2.7.5), written without TensorFlow.

The reference exports with ``export_savedmodel(servable_model_dir,
build_raw_serving_input_receiver_fn({feat_ids, feat_vals}))`` (PS:451-467): a SavedModel whose
MetaGraphDef (tag ``serve``) holds the inference graph of ``model_fn`` (PREDICT mode, PS:149-241),
a V2 SaverDef that restores ``variables/variables`` and the ``serving_default`` signature

    inputs  feat_ids  int64[-1, F]   feat_vals float32[-1, F]
    outputs prob      float32[-1]                                  (method tensorflow/serving/predict)

This module encodes that protobuf directly (field numbers of tensorflow/core/protobuf/
{saved_model,meta_graph,saver}.proto and framework/{graph,node_def,attr_value,tensor,
tensor_shape}.proto): the graph is the DeepFM forward in standard TF1 ops (Placeholder,
VariableV2 + Identity reads, GatherV2, Mul, Sum, Square, Sub, Reshape, MatMul, BiasAdd, Relu,
batch-norm inference arithmetic, Add, Sigmoid) with the reference's variable and scope names, so
the variables bundle written next to it restores by name.  Without TensorFlow the file is checked
structurally only (tests/test_ckpt.py decodes it back): TF parity is unpinned.
"""
from __future__ import annotations

import struct
from typing import Dict, List, Optional, Sequence, Tuple

from ..data.tfrecord import _varint

DT_FLOAT, DT_INT32, DT_STRING, DT_INT64 = 1, 3, 7, 9
_TF_VERSION = "1.15.2"          # the reference's framework_version (NBPS:212)
_GRAPH_PRODUCER = 134           # GraphDef version of TF 1.15


# ------------------------------------------------------------------------------ wire format
def _ld(f: int, payload: bytes) -> bytes:
    return _varint((f << 3) | 2) + _varint(len(payload)) + payload


def _vi(f: int, v: int) -> bytes:
    return _varint(f << 3) + _varint(v & 0xFFFFFFFFFFFFFFFF)


def _str(f: int, s: str) -> bytes:
    return _ld(f, s.encode())


def _f32(f: int, v: float) -> bytes:
    return _varint((f << 3) | 5) + struct.pack("<f", v)


def _map_entry(f: int, key: str, value: bytes) -> bytes:
    return _ld(f, _str(1, key) + _ld(2, value))


def shape_proto(dims: Optional[Sequence[int]]) -> bytes:
    if dims is None:
        return _vi(3, 1)                                   # unknown_rank
    return b"".join(_ld(2, _vi(1, d) if d != 0 else b"") for d in dims)


def tensor_proto(dtype: int, dims: Sequence[int], *, ints=None, int64s=None, floats=None,
                 strings=None) -> bytes:
    out = _vi(1, dtype) + _ld(2, shape_proto(dims))
    if floats is not None:
        out += _ld(5, b"".join(struct.pack("<f", x) for x in floats))
    if ints is not None:
        out += _ld(7, b"".join(_varint(x & 0xFFFFFFFFFFFFFFFF) for x in ints))
    if strings is not None:
        out += b"".join(_ld(8, s.encode()) for s in strings)
    if int64s is not None:
        out += _ld(10, b"".join(_varint(x & 0xFFFFFFFFFFFFFFFF) for x in int64s))
    return out


# AttrValue
def a_type(t: int) -> bytes:
    return _vi(6, t)


def a_shape(dims) -> bytes:
    return _ld(7, shape_proto(dims))


def a_tensor(t: bytes) -> bytes:
    return _ld(8, t)


def a_bool(b: bool) -> bytes:
    return _vi(5, 1 if b else 0)


def a_int(i: int) -> bytes:
    return _vi(3, i)


def a_str(s: str) -> bytes:
    return _str(2, s)


def a_types(ts: List[int]) -> bytes:
    return _ld(1, _ld(6, b"".join(_varint(t) for t in ts)))


def node(name: str, op: str, inputs: Sequence[str] = (), attrs: Optional[Dict[str, bytes]] = None) -> bytes:
    out = _str(1, name) + _str(2, op)
    for i in inputs:
        out += _str(3, i)
    for k in sorted(attrs or {}):
        out += _map_entry(5, k, attrs[k])
    return out


def tensor_info(name: str, dtype: int, dims) -> bytes:
    return _str(1, name) + _vi(2, dtype) + _ld(3, shape_proto(dims))


# ------------------------------------------------------------------------------ the graph
class _G:
    def __init__(self):
        self.nodes: List[bytes] = []
        self.names: List[str] = []

    def add(self, name, op, inputs=(), attrs=None) -> str:
        self.nodes.append(node(name, op, inputs, attrs))
        self.names.append(name)
        return name

    def const_i32(self, name, vals, dims) -> str:
        return self.add(name, "Const", (), {"dtype": a_type(DT_INT32),
                                           "value": a_tensor(tensor_proto(DT_INT32, dims, ints=vals))})

    def const_f32(self, name, val) -> str:
        return self.add(name, "Const", (), {"dtype": a_type(DT_FLOAT),
                                           "value": a_tensor(tensor_proto(DT_FLOAT, [], floats=[val]))})

    def var(self, name, dims, dtype=DT_FLOAT) -> str:
        self.add(name, "VariableV2", (), {"dtype": a_type(dtype), "shape": a_shape(dims),
                                          "container": a_str(""), "shared_name": a_str("")})
        return self.add(name + "/read", "Identity", (name,), {"T": a_type(dtype),
                                                              "_class": _ld(1, _ld(2, f"loc:@{name}".encode()))})


def _f(t=DT_FLOAT):
    return {"T": a_type(t)}


def serving_graph(cfg: dict) -> Tuple[List[bytes], List[Tuple[str, List[int], int]]]:
    """Nodes of the PREDICT-mode graph of the reference model_fn + the list of variables
    (name, TF shape, dtype) that the saver restores."""
    V, F, K = cfg["feature_size"], cfg["field_size"], cfg["embedding_size"]
    layers = list(cfg["deep_layers"])
    bn = bool(cfg.get("batch_norm", False))
    g = _G()
    ids = g.add("feat_ids", "Placeholder", (), {"dtype": a_type(DT_INT64), "shape": a_shape([-1, F])})
    vals = g.add("feat_vals", "Placeholder", (), {"dtype": a_type(DT_FLOAT), "shape": a_shape([-1, F])})
    variables = [("fm_bias", [1], DT_FLOAT), ("fm_w", [V], DT_FLOAT), ("fm_v", [V, K], DT_FLOAT)]
    fb, fw, fv = g.var("fm_bias", [1]), g.var("fm_w", [V]), g.var("fm_v", [V, K])
    axis0 = g.const_i32("Const/axis0", [0], [])
    one = g.const_i32("Const/axis1", [1], [])
    gat = {"Tparams": a_type(DT_FLOAT), "Tindices": a_type(DT_INT64), "Taxis": a_type(DT_INT32),
           "batch_dims": a_int(0)}
    red = {"T": a_type(DT_FLOAT), "Tidx": a_type(DT_INT32), "keep_dims": a_bool(False)}
    # first order: y_w = sum_f w[ids] * x                                    (PS:177-179)
    w = g.add("First-order/embedding_lookup", "GatherV2", (fw, ids, axis0), gat)
    wx = g.add("First-order/Mul", "Mul", (w, vals), _f())
    y_w = g.add("First-order/Sum", "Sum", (wx, one), red)
    # second order: E = v[ids] * x; y_v = 0.5 * sum_k((sum_f E)^2 - sum_f E^2)  (PS:181-187)
    emb = g.add("Second-order/embedding_lookup", "GatherV2", (fv, ids, axis0), gat)
    shp = g.const_i32("Second-order/Reshape/shape", [-1, F, 1], [3])
    xr = g.add("Second-order/Reshape", "Reshape", (vals, shp), {"T": a_type(DT_FLOAT), "Tshape": a_type(DT_INT32)})
    E = g.add("Second-order/Mul", "Mul", (emb, xr), _f())
    s = g.add("Second-order/Sum", "Sum", (E, one), red)
    s2 = g.add("Second-order/Square", "Square", (s,), _f())
    e2 = g.add("Second-order/Square_1", "Square", (E,), _f())
    q = g.add("Second-order/Sum_1", "Sum", (e2, one), red)
    d = g.add("Second-order/Sub", "Sub", (s2, q), _f())
    half = g.const_f32("Second-order/mul/x", 0.5)
    sd = g.add("Second-order/Sum_2", "Sum", (d, one), red)
    y_v = g.add("Second-order/mul", "Mul", (half, sd), _f())
    # deep tower (inference: no dropout; batch norm with moving statistics)  (PS:189-226)
    dshape = g.const_i32("Deep-part/Reshape/shape", [-1, F * K], [2])
    x = g.add("Deep-part/Reshape", "Reshape", (E, dshape), {"T": a_type(DT_FLOAT), "Tshape": a_type(DT_INT32)})
    din = F * K
    mm = {"T": a_type(DT_FLOAT), "transpose_a": a_bool(False), "transpose_b": a_bool(False)}
    for i, L in enumerate(layers):
        sc = f"Deep-part/mlp{i}"
        W = g.var(f"{sc}/weights", [din, L])
        b = g.var(f"{sc}/biases", [L])
        variables += [(f"{sc}/weights", [din, L], DT_FLOAT), (f"{sc}/biases", [L], DT_FLOAT)]
        h = g.add(f"{sc}/MatMul", "MatMul", (x, W), mm)
        h = g.add(f"{sc}/BiasAdd", "BiasAdd", (h, b), {"T": a_type(DT_FLOAT), "data_format": a_str("NHWC")})
        x = g.add(f"{sc}/Relu", "Relu", (h,), _f())
        if bn:
            bs = f"Deep-part/bn_{i}"
            beta, gamma = g.var(f"{bs}/beta", [L]), g.var(f"{bs}/gamma", [L])
            mmean, mvar = g.var(f"{bs}/moving_mean", [L]), g.var(f"{bs}/moving_variance", [L])
            variables += [(f"{bs}/{n}", [L], DT_FLOAT) for n in ("beta", "gamma", "moving_mean",
                                                                 "moving_variance")]
            eps = g.const_f32(f"{bs}/batchnorm/add/y", 1e-3)
            ve = g.add(f"{bs}/batchnorm/add", "Add", (mvar, eps), _f())
            rs = g.add(f"{bs}/batchnorm/Rsqrt", "Rsqrt", (ve,), _f())
            gm = g.add(f"{bs}/batchnorm/mul", "Mul", (rs, gamma), _f())
            xm = g.add(f"{bs}/batchnorm/mul_1", "Mul", (x, gm), _f())
            mg = g.add(f"{bs}/batchnorm/mul_2", "Mul", (mmean, gm), _f())
            sh = g.add(f"{bs}/batchnorm/sub", "Sub", (beta, mg), _f())
            x = g.add(f"{bs}/batchnorm/add_1", "Add", (xm, sh), _f())
        din = L
    Wo = g.var("Deep-part/deep_out/weights", [din, 1])
    bo = g.var("Deep-part/deep_out/biases", [1])
    variables += [("Deep-part/deep_out/weights", [din, 1], DT_FLOAT), ("Deep-part/deep_out/biases", [1], DT_FLOAT)]
    h = g.add("Deep-part/deep_out/MatMul", "MatMul", (x, Wo), mm)
    h = g.add("Deep-part/deep_out/BiasAdd", "BiasAdd", (h, bo), {"T": a_type(DT_FLOAT), "data_format": a_str("NHWC")})
    oshape = g.const_i32("Deep-part/Reshape_1/shape", [-1], [1])
    y_d = g.add("Deep-part/Reshape_1", "Reshape", (h, oshape), {"T": a_type(DT_FLOAT), "Tshape": a_type(DT_INT32)})
    # y = b + y_w + y_v + y_d, prob = sigmoid(y)                             (PS:228-232)
    y = g.add("DeepFM-out/add", "Add", (fb, y_w), _f())
    y = g.add("DeepFM-out/add_1", "Add", (y, y_v), _f())
    y = g.add("DeepFM-out/add_2", "Add", (y, y_d), _f())
    g.add("prob", "Sigmoid", (y,), _f())
    variables.append(("global_step", [], DT_INT64))
    g.add("global_step", "VariableV2", (), {"dtype": a_type(DT_INT64), "shape": a_shape([]),
                                           "container": a_str(""), "shared_name": a_str("")})
    # V2 saver: RestoreV2 of every variable from the bundle prefix fed into save/Const
    names = [v[0] for v in variables]
    dtypes = [v[2] for v in variables]
    fn = g.add("save/Const", "Const", (), {"dtype": a_type(DT_STRING),
                                         "value": a_tensor(tensor_proto(DT_STRING, [], strings=["model"]))})
    tn = g.add("save/RestoreV2/tensor_names", "Const", (), {
        "dtype": a_type(DT_STRING), "value": a_tensor(tensor_proto(DT_STRING, [len(names)], strings=names))})
    ss = g.add("save/RestoreV2/shape_and_slices", "Const", (), {
        "dtype": a_type(DT_STRING), "value": a_tensor(tensor_proto(DT_STRING, [len(names)], strings=[""] * len(names)))})
    rv = g.add("save/RestoreV2", "RestoreV2", (fn, tn, ss), {"dtypes": a_types(dtypes)})
    assigns = []
    for i, (n, _, dt) in enumerate(variables):
        src = rv if i == 0 else f"{rv}:{i}"
        assigns.append(g.add(f"save/Assign_{i}" if i else "save/Assign", "Assign", (n, src), {
            "T": a_type(dt), "use_locking": a_bool(True), "validate_shape": a_bool(True)}))
    g.add("save/restore_all", "NoOp", tuple("^" + a for a in assigns))
    sv = g.add("save/SaveV2", "SaveV2", (fn, tn, ss) + tuple(names), {"dtypes": a_types(dtypes)})
    g.add("save/control_dependency", "Identity", (fn, "^" + sv), {
        "T": a_type(DT_STRING), "_class": _ld(1, _ld(2, b"loc:@save/Const"))})
    return g.nodes, variables


def saved_model_bytes(cfg: dict) -> bytes:
    nodes, variables = serving_graph(cfg)
    F = cfg["field_size"]
    graph = b"".join(_ld(1, n) for n in nodes) + _ld(4, _vi(1, _GRAPH_PRODUCER) + _vi(2, 12))
    meta_info = _str(1, "v1") + _str(4, "serve") + _str(5, _TF_VERSION)
    saver = (_str(1, "save/Const:0") + _str(2, "save/control_dependency:0") +
             _str(3, "save/restore_all") + _vi(4, 5) + _vi(5, 1) + _f32(6, 10000.0) + _vi(7, 2))
    sig = (_map_entry(1, "feat_ids", tensor_info("feat_ids:0", DT_INT64, [-1, F])) +
           _map_entry(1, "feat_vals", tensor_info("feat_vals:0", DT_FLOAT, [-1, F])) +
           _map_entry(2, "prob", tensor_info("prob:0", DT_FLOAT, [-1])) +
           _str(3, "tensorflow/serving/predict"))
    var_names = b"".join(_str(1, n) for n, _, _ in variables)
    colls = (_map_entry(4, "variables", _ld(1, var_names)) +
             _map_entry(4, "trainable_variables",
                        _ld(1, b"".join(_str(1, n) for n, _, _ in variables
                                        if n != "global_step" and "moving_" not in n))))
    meta = (_ld(1, meta_info) + _ld(2, graph) + _ld(3, saver) + colls +
            _map_entry(5, "serving_default", sig))
    return _vi(1, 1) + _ld(2, meta)


def write_saved_model(path: str, cfg: dict) -> None:
    with open(path, "wb") as f:
        f.write(saved_model_bytes(cfg))
