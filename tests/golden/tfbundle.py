"""Minimal, dependency-free readers for the reference's TF 1.3 artefacts.

Test infrastructure only (fixture generation).  Used to decode the reference's
committed checkpoints (`results/model_ddpg/model-120.*`,
`InvertedPendulum/model_ddpg/model-1410.*`) and MetaGraphDefs into plain numpy
fixtures under tests/golden/ (SURVEY.md §4.3).  Nothing here executes anything
from the files: it is a byte-level SSTable + protobuf wire-format walker.

Formats:
  * `.index`  -- LevelDB SSTable (uncompressed).  48-byte footer
    [metaindex handle][index handle][pad][magic 0xdb4775248b80fb57]; blocks are
    prefix-compressed entries + restart array; each value is a
    `BundleEntryProto` {1 dtype, 2 shape{2 dim{1 size}}, 3 shard, 4 offset,
    5 size}.
  * `.data-00000-of-00001` -- raw little-endian tensor bytes at those offsets.
  * `.meta`   -- MetaGraphDef {1 meta_info_def{5 tf_version}, 2 graph_def
    {1 node{1 name, 2 op, 3 input, 4 device, 5 attr}}}.
"""
import struct

import numpy as np

_MAGIC = 0xDB4775248B80FB57


def _varint(buf, pos):
    result = 0
    shift = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def pb_fields(buf):
    """Yield (field_number, wire_type, value) for a protobuf message."""
    pos = 0
    n = len(buf)
    while pos < n:
        key, pos = _varint(buf, pos)
        fno, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _varint(buf, pos)
        elif wt == 1:
            v = buf[pos:pos + 8]
            pos += 8
        elif wt == 2:
            ln, pos = _varint(buf, pos)
            v = buf[pos:pos + ln]
            pos += ln
        elif wt == 5:
            v = buf[pos:pos + 4]
            pos += 4
        else:
            raise ValueError("unsupported wire type %d" % wt)
        yield fno, wt, v


def _block_entries(data, off, size):
    blk = data[off:off + size]
    nrestart = struct.unpack_from("<I", blk, len(blk) - 4)[0]
    end = len(blk) - 4 - 4 * nrestart
    pos = 0
    key = b""
    while pos < end:
        shared, pos = _varint(blk, pos)
        nonshared, pos = _varint(blk, pos)
        vlen, pos = _varint(blk, pos)
        key = key[:shared] + blk[pos:pos + nonshared]
        pos += nonshared
        val = blk[pos:pos + vlen]
        pos += vlen
        yield key, val


def read_index(path):
    """Return {tensor_name: (dtype_enum, shape_tuple, offset, size)}."""
    data = open(path, "rb").read()
    footer = data[-48:]
    magic = struct.unpack_from("<Q", footer, 40)[0]
    if magic != _MAGIC:
        raise ValueError("not an SSTable: %s" % path)
    p = 0
    _, p = _varint(footer, p)
    _, p = _varint(footer, p)  # metaindex handle (unused)
    idx_off, p = _varint(footer, p)
    idx_size, p = _varint(footer, p)
    out = {}
    for _, handle in _block_entries(data, idx_off, idx_size):
        boff, q = _varint(handle, 0)
        bsize, q = _varint(handle, q)
        for key, val in _block_entries(data, boff, bsize):
            if key == b"":
                continue  # BundleHeaderProto
            dtype, shape, offset, size = None, [], 0, 0
            for fno, wt, v in pb_fields(val):
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
                    offset = v
                elif fno == 5:
                    size = v
            out[key.decode()] = (dtype, tuple(shape), offset, size)
    return out


def read_checkpoint(prefix):
    """Decode a TF V2 bundle into {name: np.ndarray} (DT_FLOAT only)."""
    index = read_index(prefix + ".index")
    blob = open(prefix + ".data-00000-of-00001", "rb").read()
    out = {}
    for name, (dtype, shape, off, size) in index.items():
        if dtype != 1:  # DT_FLOAT
            continue
        arr = np.frombuffer(blob, dtype="<f4", count=size // 4, offset=off)
        out[name] = arr.reshape(shape).copy()
    return out


def read_meta_nodes(path):
    """Return (tf_version, [(name, op, device, {attr: raw_bytes})])."""
    data = open(path, "rb").read()
    version = None
    nodes = []
    for fno, _, v in pb_fields(data):
        if fno == 1:
            for f2, _, v2 in pb_fields(v):
                if f2 == 5:
                    version = v2.decode()
        elif fno == 2:
            for f2, _, nd in pb_fields(v):
                if f2 != 1:
                    continue
                name = op = device = ""
                attrs = {}
                for f3, _, v3 in pb_fields(nd):
                    if f3 == 1:
                        name = v3.decode()
                    elif f3 == 2:
                        op = v3.decode()
                    elif f3 == 4:
                        device = v3.decode()
                    elif f3 == 5:
                        k = val = None
                        for f4, _, v4 in pb_fields(v3):
                            if f4 == 1:
                                k = v4.decode()
                            elif f4 == 2:
                                val = v4
                        attrs[k] = val
                nodes.append((name, op, device, attrs))
    return version, nodes


def const_float(attrs):
    """Scalar float value of a Const node's `value` attr (TensorProto)."""
    av = attrs.get("value")
    if av is None:
        return None
    for fno, _, tp in pb_fields(av):  # AttrValue.tensor = 8
        if fno != 8:
            continue
        for f2, wt, v in pb_fields(tp):
            if f2 == 5:  # float_val
                if wt == 2:
                    return struct.unpack_from("<f", v, 0)[0]
                return struct.unpack("<f", v)[0]
            if f2 == 4:  # tensor_content
                if len(v) >= 4:
                    return struct.unpack_from("<f", v, 0)[0]
    return None
