"""TensorBoard scalar writer/reader, pinned on the
reference's own MountainCar event file (tests/golden/events_mc_scalars.tfrecord:
its records copied verbatim by make_events_fixture.py)."""
import os
import struct

import numpy as np

from conftest import GOLDEN

REF = os.path.join(GOLDEN, "events_mc_scalars.tfrecord")


def test_reference_event_file_decodes_with_valid_crcs():
    from distributed_ddpg_amd import summary as S
    recs = list(S.read_records(REF))  # raises on any CRC mismatch
    first = S.decode_event(recs[0])
    assert first["file_version"] == "brain.Event:2"
    sc = S.read_scalars(REF)
    assert set(S.TRAIN_TAGS) <= set(sc)
    rewards = [v for _, v in sc["Reward"]]
    assert len(rewards) == 121                          # 121 episodes
    assert abs(np.mean(rewards[-10:]) - 93.9) < 0.05    # last-10 mean 93.9
    assert abs(max(rewards) - 97.65) < 0.01             # max 97.65
    assert [s for s, _ in sc["Reward"]] == list(range(121))


def test_writer_matches_tf_record_layout(tmp_path):
    from distributed_ddpg_amd import summary as S
    ref = list(S.read_records(REF))
    # the same Event bytes TF wrote, re-encoded from their decoded fields
    for rec in ref[:6]:
        ev = S.decode_event(rec)
        again = S.encode_event(ev["wall_time"], ev["step"], ev["scalars"] or None,
                               ev["file_version"])
        assert again == rec
    # the framing of a whole record, CRCs included
    data = open(REF, "rb").read()
    (ln,) = struct.unpack_from("<Q", data, 0)
    assert S.frame(ref[0]) == data[:16 + ln]
    w = S.FileWriter(str(tmp_path / "tboard"))
    w.add_episode(0, 1.5, 0.25, 3.0)
    w.add_scalars(7, [("Validation_Rewards", 950.0)])
    w.close()
    assert os.path.basename(w.path).startswith("events.out.tfevents.")
    recs = [S.decode_event(r) for r in S.read_records(w.path)]
    assert recs[0]["file_version"] == "brain.Event:2"
    assert recs[1]["step"] == 0 and recs[1]["scalars"] == [("Reward", 1.5), ("Qmax_Value", 0.25),
                                                           ("Value_Loss", 3.0)]
    assert recs[2]["step"] == 7 and recs[2]["scalars"] == [("Validation_Rewards", 950.0)]
