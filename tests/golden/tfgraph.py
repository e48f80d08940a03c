"""A small numpy interpreter for the reference's TF 1.3 GraphDef.

Test infrastructure only (fixture generation, build container).  It decodes the
MetaGraphDef the reference saved next to its checkpoints
(`InvertedPendulum/model_ddpg/model-1410.meta`, `results/model_ddpg/model-120.meta`)
and executes the reference's own dataflow graph -- the 34 MatMuls, the
gradient subgraphs tf.gradients built (`networks.py:44, 136-137, 143`), the 13
ApplyAdam nodes and the soft-update Mul/Add/Assign nodes
(`networks.py:34-37, 126-128`) -- node by node, with session-run semantics:
every node is evaluated at most once per run (so variable reads inside one run
see the pre-update value, as in TF), control inputs (`^name`) are executed,
and Assign / ApplyAdam mutate the variable store.

What is pinned this way: the WIRING (which tensors feed which op, grad_ys,
the loss and its gradient chain, the optimiser and soft-update structure,
every graph constant).  What is NOT: the op kernels themselves, which are
restated below from TF 1.3's formulas (Elu/EluGrad from the output, TanhGrad,
ApplyAdam's epsilon-hat form, BiasAddGrad, the Mean/Square/Sub gradient
helpers).  Nothing in the file is executed: it is parsed as protobuf wire data.

Arithmetic runs in float64 (`dtype=np.float64`, graph float constants widened
from their stored float32 values) or float32.
"""
import struct

import numpy as np

from tfbundle import pb_fields

_DT = {1: np.float32, 2: np.float64, 3: np.int32, 9: np.int64, 10: np.bool_}


def _attr_value(raw):
    """Decode an AttrValue into a python value (only the kinds the graph uses)."""
    out = None
    for fno, wt, v in pb_fields(raw):
        if fno == 2:  # s
            out = bytes(v)
        elif fno == 3:  # i
            out = v
        elif fno == 4:  # f
            out = struct.unpack("<f", v)[0]
        elif fno == 5:  # b
            out = bool(v)
        elif fno == 6:  # type
            out = ("type", v)
        elif fno == 8:  # tensor
            out = ("tensor", v)
        elif fno == 7:  # shape
            out = ("shape", v)
        elif fno == 1:  # list
            out = ("list", v)
    return out


def decode_tensor(raw):
    """TensorProto -> numpy array."""
    dtype, shape, content = 1, [], None
    vals = {5: [], 6: [], 7: [], 10: [], 11: []}
    for fno, wt, v in pb_fields(raw):
        if fno == 1:
            dtype = v
        elif fno == 2:
            for f2, _, dim in pb_fields(v):
                if f2 == 2:
                    sz = 0
                    for f3, _, dv in pb_fields(dim):
                        if f3 == 1:
                            sz = dv
                    shape.append(sz)
        elif fno == 4:
            content = bytes(v)
        elif fno in vals:
            if wt == 2:  # packed
                if fno == 5:
                    vals[5].extend(struct.unpack("<%df" % (len(v) // 4), v))
                elif fno == 6:
                    vals[6].extend(struct.unpack("<%dd" % (len(v) // 8), v))
                else:
                    pos = 0
                    while pos < len(v):
                        x, pos = _varint(v, pos)
                        vals[fno].append(x)
            elif wt == 5:
                vals[fno].append(struct.unpack("<f", v)[0])
            elif wt == 1:
                vals[fno].append(struct.unpack("<d", v)[0])
            else:
                vals[fno].append(v)
    npdt = _DT[dtype]
    n = int(np.prod(shape)) if shape else 1
    if content is not None:
        arr = np.frombuffer(content, dtype=np.dtype(npdt).newbyteorder("<")).copy()
    else:
        src = {1: 5, 2: 6, 3: 7, 9: 10, 10: 11}[dtype]
        lst = vals[src]
        if npdt in (np.int32, np.int64):
            lst = [x - (1 << 64) if x >= (1 << 63) else x for x in lst]
        if n == 0:
            return np.zeros(shape, npdt)
        arr = np.array(lst if lst else [0], dtype=npdt)
        if arr.size == 1 and n > 1:
            arr = np.full(n, arr[0], npdt)
    return arr.reshape(shape)


def _varint(buf, pos):
    r, s = 0, 0
    while True:
        b = buf[pos]
        pos += 1
        r |= (b & 0x7F) << s
        if not b & 0x80:
            return r, pos
        s += 7


def read_graph(path):
    """{name: (op, [inputs], {attr: value})} of the MetaGraphDef's GraphDef."""
    data = open(path, "rb").read()
    nodes = {}
    for fno, _, v in pb_fields(data):
        if fno != 2:
            continue
        for f2, _, nd in pb_fields(v):
            if f2 != 1:
                continue
            name, op, inputs, attrs = "", "", [], {}
            for f3, _, v3 in pb_fields(nd):
                if f3 == 1:
                    name = v3.decode()
                elif f3 == 2:
                    op = v3.decode()
                elif f3 == 3:
                    inputs.append(v3.decode())
                elif f3 == 5:
                    k = val = None
                    for f4, _, v4 in pb_fields(v3):
                        if f4 == 1:
                            k = v4.decode()
                        elif f4 == 2:
                            val = v4
                    attrs[k] = _attr_value(val)
            nodes[name] = (op, inputs, attrs)
    return nodes


class Ref:
    """A variable reference (VariableV2 output, Assign / ApplyAdam result)."""

    def __init__(self, name):
        self.name = name


class Session:
    """Executes fetches of a decoded graph against a variable store."""

    def __init__(self, nodes, variables, dtype=np.float64):
        self.nodes = nodes
        self.vars = {k: np.array(v, dtype) for k, v in variables.items()}
        self.dt = np.dtype(dtype).type

    def _f(self, x):
        x = np.asarray(x)
        return x.astype(self.dt) if x.dtype.kind == "f" else x

    def run(self, fetches, feed=None):
        self._memo = {}
        self._feed = {k: self._f(v) for k, v in (feed or {}).items()}
        single = isinstance(fetches, str)
        out = [self._eval(f) for f in ([fetches] if single else fetches)]
        return out[0] if single else out

    def _eval(self, ref):
        if ref.startswith("^"):
            self._eval(ref[1:])
            return None
        name, idx = (ref.rsplit(":", 1) + ["0"])[:2] if ":" in ref else (ref, "0")
        idx = int(idx)
        if name not in self._memo:
            self._memo[name] = self._exec(name)
        v = self._memo[name]
        return v[idx] if isinstance(v, tuple) else v

    def _exec(self, name):
        if name in self._feed:
            return self._feed[name]
        op, inputs, attrs = self.nodes[name]
        data = [i for i in inputs if not i.startswith("^")]
        for c in inputs:
            if c.startswith("^"):
                self._eval(c)
        if op == "VariableV2":
            return Ref(name)
        if op == "Placeholder":
            raise KeyError("placeholder %s not fed" % name)
        if op == "Const":
            return self._f(decode_tensor(attrs["value"][1]))
        if op in ("ApplyAdam", "Assign"):
            ref = self._eval(data[0])
            assert isinstance(ref, Ref), name
            var = ref.name
        x = [self._val(self._eval(i)) for i in (data if op not in ("ApplyAdam", "Assign")
                                                  else data[1:])]
        d = self.dt
        if op == "Identity":
            return x[0]
        if op == "NoOp":
            return None
        if op == "MatMul":
            a, b = x
            if attrs.get("transpose_a"):
                a = a.T
            if attrs.get("transpose_b"):
                b = b.T
            return a @ b
        if op == "BiasAdd":
            return x[0] + x[1]
        if op == "BiasAddGrad":
            return x[0].sum(axis=0)
        if op == "Elu":  # TF: x < 0 ? exp(x) - 1 : x
            return np.where(x[0] < 0, np.exp(np.minimum(x[0], 0)) - d(1), x[0])
        if op == "EluGrad":  # EluGrad(dy, y) from the output y
            dy, y = x
            return np.where(y < 0, dy * (y + d(1)), dy)
        if op == "Tanh":
            return np.tanh(x[0])
        if op == "TanhGrad":  # TanhGrad(y, dy)
            y, dy = x
            return dy * (d(1) - y * y)
        if op == "Mul":
            return x[0] * x[1]
        if op == "Add":
            return x[0] + x[1]
        if op == "Sub":
            return x[0] - x[1]
        if op == "Neg":
            return -x[0]
        if op == "Square":
            return x[0] * x[0]
        if op == "RealDiv":
            return x[0] / x[1]
        if op == "Maximum":
            return np.maximum(x[0], x[1])
        if op == "FloorDiv":
            return x[0] // x[1]
        if op == "FloorMod":
            return np.mod(x[0], x[1])
        if op == "Cast":
            dst = _DT[attrs["DstT"][1]]
            return self._f(np.asarray(x[0]).astype(dst))
        if op == "Mean" or op == "Sum":
            axes = tuple(int(a) for a in np.atleast_1d(x[1]))
            fn = np.mean if op == "Mean" else np.sum
            return fn(x[0], axis=axes, keepdims=bool(attrs.get("keep_dims")))
        if op == "Prod":
            axes = tuple(int(a) for a in np.atleast_1d(x[1]))
            return np.prod(x[0], axis=axes, keepdims=bool(attrs.get("keep_dims"))).astype(
                x[0].dtype)
        if op == "Shape":
            return np.array(np.shape(x[0]), np.int32)
        if op == "ShapeN":
            return tuple(np.array(np.shape(v), np.int32) for v in x)
        if op == "Reshape":
            return np.reshape(x[0], [int(s) for s in np.atleast_1d(x[1])])
        if op == "Fill":
            return np.full([int(s) for s in x[0]], x[1])
        if op == "Tile":
            return np.tile(x[0], [int(s) for s in x[1]])
        if op == "ConcatV2":
            return np.concatenate(x[:-1], axis=int(x[-1]))
        if op == "ConcatOffset":
            axis, shapes = int(x[0]), x[1:]
            offs, o = [], 0
            for s in shapes:
                off = np.zeros_like(s)
                off[axis] = o
                o += int(s[axis])
                offs.append(off)
            return tuple(offs)
        if op == "Slice":
            begin = [int(b) for b in x[1]]
            size = [int(s) for s in x[2]]
            sl = tuple(slice(b, None if s == -1 else b + s) for b, s in zip(begin, size))
            return x[0][sl]
        if op == "BroadcastGradientArgs":
            s0, s1 = [int(v) for v in x[0]], [int(v) for v in x[1]]
            n = max(len(s0), len(s1))
            s0 = [1] * (n - len(s0)) + s0
            s1 = [1] * (n - len(s1)) + s1
            r0 = [i for i in range(n) if s0[i] == 1 and s1[i] != 1]
            r1 = [i for i in range(n) if s1[i] == 1 and s0[i] != 1]
            return np.array(r0, np.int32), np.array(r1, np.int32)
        if op == "Assign":
            self.vars[var] = np.array(x[0], dtype=self.vars[var].dtype).reshape(
                self.vars[var].shape)
            return Ref(var)
        if op == "ApplyAdam":
            # inputs: var, m, v, beta1_power, beta2_power, lr, beta1, beta2, epsilon, grad
            m_ref = self._eval(data[1]).name
            v_ref = self._eval(data[2]).name
            b1p, b2p, lr, b1, b2, eps, g = x[2:]
            one = d(1)
            alpha = lr * np.sqrt(one - b2p) / (one - b1p)
            m = self.vars[m_ref]
            v = self.vars[v_ref]
            m = m + (g - m) * (one - b1)
            v = v + (g * g - v) * (one - b2)
            self.vars[m_ref], self.vars[v_ref] = m, v
            self.vars[var] = self.vars[var] - (m * alpha) / (np.sqrt(v) + eps)
            return Ref(var)
        raise NotImplementedError("op %s (%s)" % (op, name))

    def _val(self, v):
        """A variable ref read as a value (TF's implicit ref -> value)."""
        if isinstance(v, Ref):
            return self.vars[v.name]
        return v
