"""TensorBoard event-file writer/reader for the episode scalars
(SURVEY.md §8(f)3).

The reference logs, per episode, `Reward`, `Qmax_Value` and `Value_Loss`
(`ddpg.py:32-53` build_summaries, `:118-125` writer.add_summary) and, per
validation, `Validation_Rewards` (`:147-151`) through `tf.summary.FileWriter`
(`ddpg.py:241`).  This module writes the same TFRecord stream so that curves
from this build and the reference's committed `results/tboard_ddpg` /
`InvertedPendulum/tboard_ddpg` runs load side by side in TensorBoard:

  file    events.out.tfevents.<unix time>.<hostname>
  record  uint64 length | uint32 masked crc32c(length) | Event | uint32 masked crc32c(Event)
  Event   {1 wall_time: double, 2 step: int64, 3 file_version: "brain.Event:2",
           5 summary: {1 value: {1 tag, 2 simple_value: float}}}

The first record is the file_version event, as TF writes it.  Graph and
MetaGraph records are not written (there is no TF graph here).
"""
import os
import socket
import struct
import time

from .checkpoint import masked_crc

FILE_VERSION = "brain.Event:2"
# build_summaries() tags (ddpg.py:32-53)
TRAIN_TAGS = ("Reward", "Qmax_Value", "Value_Loss")
VALID_TAGS = ("Validation_Rewards",)


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


def _bytes_field(fno, payload):
    return _varint((fno << 3) | 2) + _varint(len(payload)) + payload


def encode_event(wall_time, step=0, scalars=None, file_version=None):
    """Serialise one Event proto (fields in TF's order; step 0 omitted as proto3 does)."""
    out = bytes([0x09]) + struct.pack("<d", wall_time)
    if step:
        out += _varint(2 << 3) + _varint(step & 0xFFFFFFFFFFFFFFFF)
    if file_version is not None:
        out += _bytes_field(3, file_version.encode())
    if scalars:
        vals = b""
        for tag, v in scalars:
            val = _bytes_field(1, tag.encode()) + bytes([(2 << 3) | 5]) + struct.pack("<f", v)
            vals += _bytes_field(1, val)
        out += _bytes_field(5, vals)
    return out


def frame(record):
    """TFRecord framing of one serialised record."""
    hdr = struct.pack("<Q", len(record))
    return hdr + struct.pack("<I", masked_crc(hdr)) + record + struct.pack("<I", masked_crc(record))


def read_records(path, verify=True):
    """Yield the serialised records of a TFRecord file (CRCs checked)."""
    data = open(path, "rb").read()
    pos = 0
    while pos < len(data):
        hdr = data[pos:pos + 8]
        (ln,) = struct.unpack("<Q", hdr)
        if verify and struct.unpack_from("<I", data, pos + 8)[0] != masked_crc(hdr):
            raise ValueError("%s: length checksum mismatch at %d" % (path, pos))
        rec = data[pos + 12:pos + 12 + ln]
        if verify and struct.unpack_from("<I", data, pos + 12 + ln)[0] != masked_crc(rec):
            raise ValueError("%s: record checksum mismatch at %d" % (path, pos))
        yield rec
        pos += 16 + ln


def _read_varint(buf, pos):
    result = shift = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def _fields(buf):
    pos = 0
    while pos < len(buf):
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
            raise ValueError("unsupported wire type %d" % wt)
        yield fno, wt, v


def decode_event(rec):
    """-> dict(wall_time, step, file_version, scalars=[(tag, value)], other=[field numbers])."""
    ev = {"wall_time": 0.0, "step": 0, "file_version": None, "scalars": [], "other": []}
    for fno, _, v in _fields(rec):
        if fno == 1:
            ev["wall_time"] = struct.unpack("<d", v)[0]
        elif fno == 2:
            ev["step"] = v
        elif fno == 3:
            ev["file_version"] = v.decode()
        elif fno == 5:
            for f2, _, val in _fields(v):
                if f2 != 1:
                    continue
                tag, sv = None, None
                for f3, _, x in _fields(val):
                    if f3 == 1:
                        tag = x.decode()
                    elif f3 == 2:
                        sv = struct.unpack("<f", x)[0]
                if tag is not None and sv is not None:
                    ev["scalars"].append((tag, sv))
        else:
            ev["other"].append(fno)  # graph_def (4), meta_graph_def (9), ...
    return ev


def read_scalars(path):
    """{tag: [(step, value), ...]} from an event file (the curves of `results/`)."""
    out = {}
    for rec in read_records(path):
        ev = decode_event(rec)
        for tag, v in ev["scalars"]:
            out.setdefault(tag, []).append((ev["step"], v))
    return out


class FileWriter:
    """tf.summary.FileWriter work-alike for scalar summaries (ddpg.py:241)."""

    def __init__(self, logdir, filename_suffix=""):
        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(logdir, "events.out.tfevents.%d.%s%s" % (
            int(time.time()), socket.gethostname(), filename_suffix))
        self._f = open(self.path, "wb")
        self._f.write(frame(encode_event(time.time(), file_version=FILE_VERSION)))

    def add_scalars(self, step, scalars):
        """One Event with a Summary of (tag, value) pairs, as writer.add_summary
        of the merged summary op does (ddpg.py:118-125)."""
        self._f.write(frame(encode_event(time.time(), int(step),
                                         [(t, float(v)) for t, v in scalars])))

    def add_episode(self, step, reward, qmax, loss):
        self.add_scalars(step, zip(TRAIN_TAGS, (reward, qmax, loss)))

    def flush(self):
        self._f.flush()

    def close(self):
        if self._f:
            self._f.close()
            self._f = None
