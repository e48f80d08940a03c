"""Extract the scalar records of the reference's MountainCar TensorBoard run
(results/tboard_ddpg/events.out.tfevents.1504605950.oreo, written by TF 1.3's
FileWriter, ddpg.py:241) into tests/golden/events_mc_scalars.tfrecord.

Records are copied byte for byte with their original TFRecord framing (length,
masked CRCs); only the two large graph records (GraphDef, MetaGraphDef) are
dropped to keep the fixture small.  Run in the build container:
    python tests/golden/make_events_fixture.py
"""
import glob
import os
import struct

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = glob.glob("/root/reference/results/tboard_ddpg/events.out.tfevents.*")[0]


def main():
    data = open(SRC, "rb").read()
    out = bytearray()
    pos = n = kept = 0
    while pos < len(data):
        (ln,) = struct.unpack_from("<Q", data, pos)
        rec = data[pos + 12:pos + 12 + ln]
        # Event field 4 (graph_def, tag 0x22) / 9 (meta_graph_def, tag 0x4a) after wall_time
        big = len(rec) > 9 and rec[9] in (0x22, 0x4A)
        if not big:
            out += data[pos:pos + 16 + ln]
            kept += 1
        pos += 16 + ln
        n += 1
    open(os.path.join(HERE, "events_mc_scalars.tfrecord"), "wb").write(bytes(out))
    print("kept %d of %d records, %d bytes" % (kept, n, len(out)))


if __name__ == "__main__":
    main()
