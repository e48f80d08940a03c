"""TF 1.x V2 checkpoint ("tensor bundle") reader/writer and a tf.train.Saver
work-alike for the learner state.

The reference saves every global variable with `tf.train.Saver(max_to_keep=5)`
(`ddpg.py:211`), `saver.save(sess, save_dir + "/model", global_step=...)`
(`ddpg.py:155-159`) and restores with
`saver.restore(sess, tf.train.latest_checkpoint(save_dir))` (`ddpg.py:213-222`).
This module writes and reads the same files with the same variable names, so a
reference checkpoint (e.g. `results/model_ddpg/model-120`) loads into this
build and a checkpoint written here loads into TF 1.3:

  <prefix>.index                 LevelDB SSTable: key "" -> BundleHeaderProto,
                                 key <var name> -> BundleEntryProto
  <prefix>.data-00000-of-00001   the tensors' little-endian bytes, key order
  checkpoint                     CheckpointState text proto (latest + kept list)

Byte-for-byte the writer reproduces TF 1.3's own output: one data block with a
restart point every 16 keys, the shortest-successor index key, an empty
metaindex block, masked-CRC32C block trailers and entry checksums (the test
suite rewrites the reference's `model-120` and compares bytes).  `.meta`
MetaGraphDefs are not written (no TF graph exists here).

Variable names (tf.trainable_variables() order, `networks.py:27,31,119,122`):
actor `FullyConnected{,_1,_2}`, actor target `_3.._5`, critic `_6.._9`
(state branch, action branch, hidden, out), critic target `_10.._13`; Adam
slots `<var>/Adam` (m) and `<var>/Adam_1` (v) of the online networks;
`beta1_power`/`beta2_power` (actor) and `beta1_power_1`/`beta2_power_1`
(critic); `global_step`, the summary `Variable`..`Variable_3` and
`is_training` are carried along as the reference's Saver does.
"""
import os
import re
import struct
from collections import OrderedDict

import numpy as np

from . import _lib

# ---------------------------------------------------------------- names
ACTOR = ("FullyConnected/W", "FullyConnected/b", "FullyConnected_1/W", "FullyConnected_1/b",
         "FullyConnected_2/W")
ACTOR_TARGET = ("FullyConnected_3/W", "FullyConnected_3/b", "FullyConnected_4/W",
                "FullyConnected_4/b", "FullyConnected_5/W")
CRITIC = ("FullyConnected_6/W", "FullyConnected_6/b", "FullyConnected_7/W", "FullyConnected_7/b",
          "FullyConnected_8/W", "FullyConnected_8/b", "FullyConnected_9/W", "FullyConnected_9/b")
CRITIC_TARGET = ("FullyConnected_10/W", "FullyConnected_10/b", "FullyConnected_11/W",
                 "FullyConnected_11/b", "FullyConnected_12/W", "FullyConnected_12/b",
                 "FullyConnected_13/W", "FullyConnected_13/b")
SUMMARY_VARS = ("Variable", "Variable_1", "Variable_2", "Variable_3")  # ddpg.py:32-53

# TF DataType enum values (types.proto)
_DT = {np.dtype("float32"): 1, np.dtype("float64"): 2, np.dtype("int32"): 3,
       np.dtype("int64"): 9, np.dtype("bool"): 10}
_NP = {v: k for k, v in _DT.items()}

_MAGIC = 0xDB4775248B80FB57
_RESTART_INTERVAL = 16

# ---------------------------------------------------------------- crc32c
def crc32c(data, crc=0):
    """CRC-32C (Castagnoli) of bytes, continuing from crc (library, slicing-by-8)."""
    buf = bytes(data)
    return int(_lib.lib.ddpg_crc32c(crc, buf, len(buf)))


def masked_crc(data):
    """LevelDB's masked CRC32C (rotate right 15, add 0xa282ead8)."""
    c = crc32c(data)
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


# ---------------------------------------------------------------- protobuf wire helpers
def _varint(n):
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf, pos):
    result = shift = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def _field_varint(fno, v):
    return _varint(fno << 3) + _varint(v)


def _field_bytes(fno, payload):
    return _varint((fno << 3) | 2) + _varint(len(payload)) + payload


def _fields(buf):
    pos, n = 0, len(buf)
    while pos < n:
        key, pos = _read_varint(buf, pos)
        fno, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _read_varint(buf, pos)
        elif wt == 1:
            v, pos = buf[pos:pos + 8], pos + 8
        elif wt == 2:
            ln, pos = _read_varint(buf, pos)
            v, pos = buf[pos:pos + ln], pos + ln
        elif wt == 5:
            v, pos = buf[pos:pos + 4], pos + 4
        else:
            raise ValueError("unsupported protobuf wire type %d" % wt)
        yield fno, wt, v


def _entry_proto(dtype, shape, offset, size, crc):
    """BundleEntryProto {1 dtype, 2 shape, 3 shard_id, 4 offset, 5 size, 6 crc32c}."""
    shp = b"".join(_field_bytes(2, _field_varint(1, d) if d else b"") for d in shape)
    out = _field_varint(1, dtype) + _field_bytes(2, shp)
    if offset:
        out += _field_varint(4, offset)
    if size:
        out += _field_varint(5, size)
    return out + bytes([(6 << 3) | 5]) + struct.pack("<I", crc)


def _header_proto():
    """BundleHeaderProto {1 num_shards = 1, 2 endianness = LITTLE, 3 version {1 producer = 1}}."""
    return _field_varint(1, 1) + _field_bytes(3, _field_varint(1, 1))


# ---------------------------------------------------------------- SSTable
def _block(entries):
    """LevelDB block: prefix-compressed entries, restart every 16 keys."""
    out = bytearray()
    restarts = []
    prev = b""
    for i, (k, v) in enumerate(entries):
        if i % _RESTART_INTERVAL == 0:
            restarts.append(len(out))
            shared = 0
        else:
            shared = 0
            while shared < min(len(prev), len(k)) and prev[shared] == k[shared]:
                shared += 1
        out += _varint(shared) + _varint(len(k) - shared) + _varint(len(v))
        out += k[shared:] + v
        prev = k
    if not restarts:
        restarts.append(0)
    for r in restarts:
        out += struct.pack("<I", r)
    out += struct.pack("<I", len(restarts))
    return bytes(out)


def _with_trailer(block):
    """Block + 5-byte trailer: compression type 0 and the masked CRC32C."""
    return block + b"\x00" + struct.pack("<I", masked_crc(block + b"\x00"))


def _short_successor(key):
    """LevelDB BytewiseComparator::FindShortSuccessor."""
    for i, b in enumerate(key):
        if b != 0xFF:
            return key[:i] + bytes([b + 1])
    return key


def _blocks(data, off, size):
    blk = data[off:off + size]
    nrestart = struct.unpack_from("<I", blk, len(blk) - 4)[0]
    end = len(blk) - 4 - 4 * nrestart
    pos, key = 0, b""
    while pos < end:
        shared, pos = _read_varint(blk, pos)
        nonshared, pos = _read_varint(blk, pos)
        vlen, pos = _read_varint(blk, pos)
        key = key[:shared] + blk[pos:pos + nonshared]
        pos += nonshared
        yield key, blk[pos:pos + vlen]
        pos += vlen


# ---------------------------------------------------------------- bundle I/O
def write_bundle(prefix, tensors):
    """Write {name: ndarray} as a TF V2 bundle at `prefix` (.index + .data-00000-of-00001).

    Tensors are laid out in key order, as TF's BundleWriter does for a Saver
    that adds variables sorted by name."""
    names = sorted(tensors, key=lambda s: s.encode())
    data = bytearray()
    entries = [(b"", _header_proto())]
    for name in names:
        arr = np.array(tensors[name], order="C", copy=True)  # keeps 0-d shapes (ascontiguousarray would not)
        dt = _DT.get(arr.dtype)
        if dt is None:
            raise TypeError("unsupported dtype %s for %s" % (arr.dtype, name))
        raw = arr.astype(arr.dtype.newbyteorder("<"), copy=False).tobytes()
        crc = masked_crc(raw)
        entries.append((name.encode(), _entry_proto(dt, arr.shape, len(data), len(raw), crc)))
        data += raw
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(prefix + ".data-00000-of-00001", "wb") as f:
        f.write(bytes(data))
    blk = _block(entries)
    out = bytearray(_with_trailer(blk))
    data_handle = _varint(0) + _varint(len(blk))
    meta = _block([])
    meta_off = len(out)
    out += _with_trailer(meta)
    index = _block([(_short_successor(entries[-1][0]), data_handle)])
    index_off = len(out)
    out += _with_trailer(index)
    footer = _varint(meta_off) + _varint(len(meta)) + _varint(index_off) + _varint(len(index))
    footer += b"\x00" * (40 - len(footer)) + struct.pack("<Q", _MAGIC)
    out += footer
    with open(prefix + ".index", "wb") as f:
        f.write(bytes(out))


def read_bundle(prefix, verify=True):
    """Read a TF V2 bundle into an OrderedDict {name: ndarray} (key order).

    verify: check every block trailer and every entry's masked CRC32C, as TF's
    BundleReader does; a mismatch raises ValueError."""
    idx = open(prefix + ".index", "rb").read()
    if struct.unpack_from("<Q", idx, len(idx) - 8)[0] != _MAGIC:
        raise ValueError("%s.index is not an SSTable" % prefix)
    footer = idx[-48:]
    p = 0
    _, p = _read_varint(footer, p)
    _, p = _read_varint(footer, p)
    ioff, p = _read_varint(footer, p)
    isize, p = _read_varint(footer, p)
    blob = open(prefix + ".data-00000-of-00001", "rb").read()
    out = OrderedDict()

    def check_trailer(off, size):
        if verify:
            want = struct.unpack_from("<I", idx, off + size + 1)[0]
            if masked_crc(idx[off:off + size + 1]) != want:
                raise ValueError("%s.index: block checksum mismatch" % prefix)

    check_trailer(ioff, isize)
    for _, handle in _blocks(idx, ioff, isize):
        boff, q = _read_varint(handle, 0)
        bsize, _ = _read_varint(handle, q)
        check_trailer(boff, bsize)
        for key, val in _blocks(idx, boff, bsize):
            if key == b"":
                continue  # BundleHeaderProto
            dtype, shape, offset, size, crc = 1, [], 0, 0, None
            for fno, _, v in _fields(val):
                if fno == 1:
                    dtype = v
                elif fno == 2:
                    for f2, _, dim in _fields(v):
                        if f2 == 2:
                            sz = 0
                            for f3, _, dv in _fields(dim):
                                if f3 == 1:
                                    sz = dv
                            shape.append(sz)
                elif fno == 4:
                    offset = v
                elif fno == 5:
                    size = v
                elif fno == 6:
                    crc = struct.unpack("<I", v)[0]
            raw = blob[offset:offset + size]
            if verify and crc is not None and masked_crc(raw) != crc:
                raise ValueError("%s: checksum mismatch for %s" % (prefix, key.decode()))
            dt = _NP.get(dtype)
            if dt is None:
                raise TypeError("unsupported dtype enum %d for %s" % (dtype, key.decode()))
            out[key.decode()] = np.frombuffer(raw, dtype=dt.newbyteorder("<")).astype(
                dt).reshape(shape)
    return out


# ---------------------------------------------------------------- CheckpointState
def _write_state(save_dir, latest, kept):
    lines = ['model_checkpoint_path: "%s"' % latest]
    lines += ['all_model_checkpoint_paths: "%s"' % k for k in kept]
    with open(os.path.join(save_dir, "checkpoint"), "w") as f:
        f.write("\n".join(lines) + "\n")


def _read_state(save_dir):
    path = os.path.join(save_dir, "checkpoint")
    if not os.path.exists(path):
        return None, []
    latest, kept = None, []
    for line in open(path):
        m = re.match(r'\s*(model_checkpoint_path|all_model_checkpoint_paths):\s*"(.*)"', line)
        if m:
            if m.group(1) == "model_checkpoint_path":
                latest = m.group(2)
            else:
                kept.append(m.group(2))
    return latest, kept


def latest_checkpoint(save_dir):
    """tf.train.latest_checkpoint: the prefix named by `<save_dir>/checkpoint`."""
    latest, _ = _read_state(save_dir)
    if latest is None:
        return None
    return latest if os.path.isabs(latest) else os.path.join(save_dir, latest)


# ---------------------------------------------------------------- learner state <-> names
def session_tensors(sess, global_step=0, summary_values=(0.0, 0.0, 0.0, 0.0)):
    """Every variable the reference's Saver writes, from a networks.Session."""
    t = OrderedDict()
    for which, names in ((_lib.ACTOR, ACTOR), (_lib.ACTOR_TARGET, ACTOR_TARGET),
                         (_lib.CRITIC, CRITIC), (_lib.CRITIC_TARGET, CRITIC_TARGET)):
        for n, v in zip(names, sess.get_params(which)):
            t[n] = np.asarray(v, dtype=np.float32)
    for (wm, wv), names in (((_lib.ACTOR_ADAM_M, _lib.ACTOR_ADAM_V), ACTOR),
                            ((_lib.CRITIC_ADAM_M, _lib.CRITIC_ADAM_V), CRITIC)):
        for n, m, v in zip(names, sess.get_params(wm), sess.get_params(wv)):
            t[n + "/Adam"] = np.asarray(m, dtype=np.float32)
            t[n + "/Adam_1"] = np.asarray(v, dtype=np.float32)
    for net, sfx in ((0, ""), (1, "_1")):
        b1p, b2p = sess.get_adam_powers(net)
        t["beta1_power" + sfx] = np.array(b1p, dtype=np.float32)
        t["beta2_power" + sfx] = np.array(b2p, dtype=np.float32)
    for n, v in zip(SUMMARY_VARS, summary_values):
        t[n] = np.array(v, dtype=np.float32)
    t["global_step"] = np.array(global_step, dtype=np.float32)
    t["is_training"] = np.array(False)
    return t


def load_session_tensors(sess, tensors, adam=True):
    """Inverse of session_tensors (Saver.restore); missing Adam slots stay as they are."""
    for which, names in ((_lib.ACTOR, ACTOR), (_lib.ACTOR_TARGET, ACTOR_TARGET),
                         (_lib.CRITIC, CRITIC), (_lib.CRITIC_TARGET, CRITIC_TARGET)):
        missing = [n for n in names if n not in tensors]
        if missing:
            raise KeyError("checkpoint lacks %s" % ", ".join(missing))
        sess.set_params(which, [np.asarray(tensors[n], dtype=np.float32) for n in names])
    if not adam:
        return
    for (wm, wv), names in (((_lib.ACTOR_ADAM_M, _lib.ACTOR_ADAM_V), ACTOR),
                            ((_lib.CRITIC_ADAM_M, _lib.CRITIC_ADAM_V), CRITIC)):
        if all(n + "/Adam" in tensors and n + "/Adam_1" in tensors for n in names):
            sess.set_params(wm, [np.asarray(tensors[n + "/Adam"], np.float32) for n in names])
            sess.set_params(wv, [np.asarray(tensors[n + "/Adam_1"], np.float32) for n in names])
    for net, sfx in ((0, ""), (1, "_1")):
        if "beta1_power" + sfx in tensors and "beta2_power" + sfx in tensors:
            sess.set_adam_powers(net, float(tensors["beta1_power" + sfx]),
                                 float(tensors["beta2_power" + sfx]))


class Saver:
    """tf.train.Saver(max_to_keep=5) work-alike over a networks.Session
    (`ddpg.py:155-159, 211-222`)."""

    def __init__(self, max_to_keep=5):
        self.max_to_keep = max_to_keep

    def save(self, sess, save_path, global_step=None, summary_values=(0.0, 0.0, 0.0, 0.0)):
        step = 0 if global_step is None else int(global_step)
        prefix = save_path if global_step is None else "%s-%d" % (save_path, step)
        write_bundle(prefix, session_tensors(sess, step, summary_values))
        save_dir = os.path.dirname(prefix) or "."
        name = os.path.basename(prefix)
        _, kept = _read_state(save_dir)
        kept = [k for k in kept if k != name] + [name]
        while self.max_to_keep and len(kept) > self.max_to_keep:
            old = kept.pop(0)
            for ext in (".index", ".data-00000-of-00001", ".meta"):
                p = os.path.join(save_dir, old + ext)
                if os.path.exists(p):
                    os.remove(p)
        _write_state(save_dir, name, kept)
        return prefix

    def restore(self, sess, save_path):
        tensors = read_bundle(save_path)
        load_session_tensors(sess, tensors)
        return tensors
