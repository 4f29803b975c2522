"""A minimal ONNX reader and numpy evaluator (TEST INFRASTRUCTURE for tests/test_kinfer.py).

Neither `onnx` nor `onnxruntime` is installed here, so the exported `.kinfer` graphs are checked
with this independent reader: a protobuf wire-format decoder for the ModelProto fields of the
ONNX IR (onnx/onnx.proto: ModelProto, GraphProto, NodeProto, AttributeProto, TensorProto,
ValueInfoProto, TypeProto) and a float32 numpy interpreter for the standard ops those graphs use.
An unknown op raises, so a graph the interpreter does not fully understand cannot pass.
"""

from __future__ import annotations

import struct

import numpy as np


def _varint(b: bytes, i: int) -> tuple[int, int]:
    v = s = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return v, i


def fields(b: bytes) -> list[tuple[int, int, object]]:
    """(field number, wire type, value) triples of one message."""
    out, i = [], 0
    while i < len(b):
        key, i = _varint(b, i)
        fn, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(b, i)
        elif wt == 1:
            v = b[i:i + 8]
            i += 8
        elif wt == 2:
            n, i = _varint(b, i)
            v = b[i:i + n]
            i += n
        elif wt == 5:
            v = b[i:i + 4]
            i += 4
        else:
            raise ValueError(f"wire type {wt}")
        out.append((fn, wt, v))
    return out


def _packed_varints(v, wt) -> list[int]:
    if wt == 0:
        return [v]
    out, i = [], 0
    while i < len(v):
        x, i = _varint(v, i)
        out.append(x)
    return out


def _signed(x: int) -> int:
    return x - (1 << 64) if x >= 1 << 63 else x


_DT = {1: np.float32, 6: np.int32, 7: np.int64, 9: np.bool_, 11: np.float64}


def tensor(b: bytes) -> tuple[str, np.ndarray]:
    dims, dt, name, raw, fdata, idata = [], 1, "", None, [], []
    for fn, wt, v in fields(b):
        if fn == 1:
            dims += [_signed(x) for x in _packed_varints(v, wt)]
        elif fn == 2:
            dt = v
        elif fn == 8:
            name = v.decode()
        elif fn == 9:
            raw = v
        elif fn == 4:
            fdata += list(struct.unpack(f"<{len(v) // 4}f", v)) if wt == 2 else list(struct.unpack("<f", v))
        elif fn == 7:
            idata += [_signed(x) for x in _packed_varints(v, wt)]
    if dt not in _DT:
        raise ValueError(f"tensor {name}: data type {dt}")
    if raw is not None:
        a = np.frombuffer(raw, dtype=_DT[dt]).copy()
    elif fdata:
        a = np.array(fdata, dtype=_DT[dt])
    else:
        a = np.array(idata, dtype=_DT[dt])
    return name, a.reshape(dims)


def attribute(b: bytes) -> tuple[str, object]:
    name, val, ints, floats = "", None, [], []
    for fn, wt, v in fields(b):
        if fn == 1:
            name = v.decode()
        elif fn == 2:
            val = struct.unpack("<f", v)[0]
        elif fn == 3:
            val = _signed(v)
        elif fn == 4:
            val = v
        elif fn == 5:
            val = tensor(v)[1]
        elif fn == 7:
            floats += list(struct.unpack(f"<{len(v) // 4}f", v)) if wt == 2 else list(struct.unpack("<f", v))
        elif fn == 8:
            ints += [_signed(x) for x in _packed_varints(v, wt)]
    if val is None:
        val = ints if ints else floats
    return name, val


def value_info(b: bytes) -> tuple[str, list]:
    name, shape = "", []
    for fn, _, v in fields(b):
        if fn == 1:
            name = v.decode()
        elif fn == 2:
            for fn2, _, tt in fields(v):
                if fn2 == 1:
                    for fn3, _, sh in fields(tt):
                        if fn3 == 2:
                            for fn4, _, d in fields(sh):
                                if fn4 == 1:
                                    dv = [x for f5, _, x in fields(d) if f5 == 1]
                                    shape.append(dv[0] if dv else None)
    return name, shape


class Model:
    def __init__(self, blob: bytes):
        self.opset = {}
        self.nodes, self.init, self.inputs, self.outputs = [], {}, [], []
        graph = None
        for fn, _, v in fields(blob):
            if fn == 7:
                graph = v
            elif fn == 8:
                f = {a: b for a, _, b in fields(v)}
                self.opset[f.get(1, b"").decode()] = f.get(2)
        if graph is None:
            raise ValueError("no graph")
        for fn, _, v in fields(graph):
            if fn == 1:
                node = {"input": [], "output": [], "op": "", "attr": {}}
                for f2, _, x in fields(v):
                    if f2 == 1:
                        node["input"].append(x.decode())
                    elif f2 == 2:
                        node["output"].append(x.decode())
                    elif f2 == 4:
                        node["op"] = x.decode()
                    elif f2 == 5:
                        k, a = attribute(x)
                        node["attr"][k] = a
                self.nodes.append(node)
            elif fn == 5:
                k, a = tensor(v)
                self.init[k] = a
            elif fn == 11:
                self.inputs.append(value_info(v))
            elif fn == 12:
                self.outputs.append(value_info(v))
        # graph inputs that are initializers (older IR) are not runtime inputs
        self.inputs = [(n, s) for n, s in self.inputs if n not in self.init]

    @property
    def ops(self) -> set[str]:
        return {n["op"] for n in self.nodes}

    def run(self, feeds: dict) -> list[np.ndarray]:
        env = dict(self.init)
        env.update({k: np.asarray(v) for k, v in feeds.items()})
        env[""] = None
        for node in self.nodes:
            args = [env[i] if i else None for i in node["input"]]
            res = _OPS[node["op"]](node["attr"], *args)
            if not isinstance(res, tuple):
                res = (res,)
            for name, r in zip(node["output"], res):
                env[name] = r
        return [env[n] for n, _ in self.outputs]


def _f32(x):
    return np.asarray(x).astype(np.float32) if np.asarray(x).dtype == np.float64 else np.asarray(x)


def _slice(a, x, starts, ends, axes=None, steps=None):
    starts, ends = list(starts), list(ends)
    axes = list(range(len(starts))) if axes is None else [int(v) % x.ndim for v in axes]
    steps = [1] * len(starts) if steps is None else list(steps)
    sl = [slice(None)] * x.ndim
    for s, e, ax, st in zip(starts, ends, axes, steps):
        n = x.shape[ax]
        s = max(min(int(s), n), -n - 1) if int(s) < 0 else min(int(s), n)
        e = int(min(max(int(e), -n - 1), n))
        sl[ax] = slice(s, e, int(st))
    return x[tuple(sl)]


def _gather(a, x, idx):
    return np.take(x, idx.astype(np.int64), axis=int(a.get("axis", 0)))


def _argmax(a, x):
    ax = int(a.get("axis", 0))
    r = np.argmax(x, axis=ax)  # first maximal index, as ONNX with select_last_index = 0
    if int(a.get("select_last_index", 0)):
        raise ValueError("select_last_index")
    return np.expand_dims(r, ax).astype(np.int64) if int(a.get("keepdims", 1)) else r.astype(np.int64)


def _reduce_sum(a, x, axes=None):
    if axes is None:
        axes = a.get("axes")
    keep = bool(int(a.get("keepdims", 1)))
    if axes is None or len(axes) == 0:
        return np.sum(x, keepdims=keep, dtype=x.dtype) if not int(a.get("noop_with_empty_axes", 0)) else x
    return np.sum(x, axis=tuple(int(v) for v in axes), keepdims=keep, dtype=x.dtype)


def _reshape(a, x, shape):
    shape = [int(s) for s in shape]
    shape = [x.shape[i] if s == 0 else s for i, s in enumerate(shape)]
    return x.reshape(shape)


def _unsqueeze(a, x, axes=None):
    axes = a.get("axes") if axes is None else axes
    for ax in sorted(int(v) % (x.ndim + len(axes)) for v in axes):
        x = np.expand_dims(x, ax)
    return x


def _squeeze(a, x, axes=None):
    axes = a.get("axes") if axes is None else axes
    return np.squeeze(x, axis=None if axes is None else tuple(int(v) for v in axes))


def _const(a):
    if "value" in a:
        return a["value"]
    if "value_float" in a:
        return np.array(a["value_float"], dtype=np.float32)
    if "value_int" in a:
        return np.array(a["value_int"], dtype=np.int64)
    if "value_ints" in a:
        return np.array(a["value_ints"], dtype=np.int64)
    raise ValueError(f"Constant {list(a)}")


def _const_of_shape(a, shape):
    v = a.get("value", np.zeros(1, np.float32))
    return np.full([int(s) for s in shape], v.ravel()[0], dtype=v.dtype)


def _cast(a, x):
    return x.astype(_DT[int(a["to"])])


def _gather_elements(a, x, idx):
    return np.take_along_axis(x, idx.astype(np.int64), axis=int(a.get("axis", 0)))


def _where(a, c, x, y):
    return np.where(c, x, y).astype(np.result_type(x, y))


def _sigmoid(a, x):
    return (1.0 / (1.0 + np.exp(-x.astype(np.float64)))).astype(np.float32)


_OPS = {
    "Constant": _const,
    "Identity": lambda a, x: x,
    "Add": lambda a, x, y: x + y,
    "Sub": lambda a, x, y: x - y,
    "Mul": lambda a, x, y: x * y,
    "Div": lambda a, x, y: x / y,
    "Neg": lambda a, x: -x,
    "Sqrt": lambda a, x: np.sqrt(x),
    "Cos": lambda a, x: np.cos(x),
    "Sin": lambda a, x: np.sin(x),
    "Tanh": lambda a, x: np.tanh(x),
    "Sigmoid": _sigmoid,
    "MatMul": lambda a, x, y: _f32(np.matmul(x.astype(np.float64), y.astype(np.float64))),
    "Less": lambda a, x, y: x < y,
    "Where": _where,
    "Concat": lambda a, *xs: np.concatenate(xs, axis=int(a["axis"])),
    "Slice": lambda a, x, s, e, ax=None, st=None: _slice(a, x, s, e, ax, st),
    "Gather": _gather,
    "GatherElements": _gather_elements,
    "ArgMax": _argmax,
    "ReduceSum": _reduce_sum,
    "Reshape": _reshape,
    "Unsqueeze": _unsqueeze,
    "Squeeze": _squeeze,
    "ConstantOfShape": _const_of_shape,
    "Shape": lambda a, x: np.array(x.shape, dtype=np.int64),
    "Cast": _cast,
    "Expand": lambda a, x, s: np.broadcast_to(x, np.broadcast_shapes(x.shape, tuple(int(v) for v in s))).copy(),
}
