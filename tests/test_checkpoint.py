"""TF V2 checkpoint reader/writer and Saver work-alike.

Pinned against the reference's own artefact: tests/golden/ckpt/model-120.* is
the reference's committed MountainCar checkpoint (results/model_ddpg/, written
by TF 1.3's tf.train.Saver, ddpg.py:155-159), kept here as data.  Reading it
and writing it back must reproduce TF's bytes exactly."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

REF = os.path.join(GOLDEN, "ckpt", "model-120")


def test_crc32c_known_answer():
    from distributed_ddpg_amd import checkpoint as C
    assert C.crc32c(b"123456789") == 0xE3069283      # RFC 3720 check value
    assert C.crc32c(b"") == 0
    assert C.crc32c(b"6789", C.crc32c(b"12345")) == 0xE3069283


def test_reference_checkpoint_rewrites_byte_exact(tmp_path):
    from distributed_ddpg_amd import checkpoint as C
    t = C.read_bundle(REF)
    assert len(t) == 62
    assert t["FullyConnected/W"].shape == (2, 48) and t["FullyConnected_8/W"].shape == (96, 128)
    assert t["is_training"].dtype == np.bool_
    out = str(tmp_path / "model-120")
    C.write_bundle(out, t)
    for ext in (".index", ".data-00000-of-00001"):
        assert open(out + ext, "rb").read() == open(REF + ext, "rb").read(), ext


def test_reference_checkpoint_matches_decoded_fixture():
    from distributed_ddpg_amd import checkpoint as C
    t = C.read_bundle(REF)
    z = np.load(os.path.join(GOLDEN, "mc_model120.npz"))
    for k in z.files:
        if k in t:
            np.testing.assert_array_equal(t[k], z[k])


def test_corruption_is_detected(tmp_path):
    from distributed_ddpg_amd import checkpoint as C
    t = C.read_bundle(REF)
    out = str(tmp_path / "m")
    C.write_bundle(out, t)
    data = bytearray(open(out + ".data-00000-of-00001", "rb").read())
    data[100] ^= 0x40
    open(out + ".data-00000-of-00001", "wb").write(bytes(data))
    with pytest.raises(ValueError, match="checksum"):
        C.read_bundle(out)
    C.read_bundle(out, verify=False)  # explicit opt-out still decodes


class _FakeSession:
    """Duck-typed networks.Session: the Saver's name mapping without a GPU."""

    def __init__(self, t):
        from distributed_ddpg_amd import _lib, checkpoint as C
        self.p = {_lib.ACTOR: [t[n] for n in C.ACTOR], _lib.ACTOR_TARGET: [t[n] for n in C.ACTOR_TARGET],
                  _lib.CRITIC: [t[n] for n in C.CRITIC],
                  _lib.CRITIC_TARGET: [t[n] for n in C.CRITIC_TARGET],
                  _lib.ACTOR_ADAM_M: [t[n + "/Adam"] for n in C.ACTOR],
                  _lib.ACTOR_ADAM_V: [t[n + "/Adam_1"] for n in C.ACTOR],
                  _lib.CRITIC_ADAM_M: [t[n + "/Adam"] for n in C.CRITIC],
                  _lib.CRITIC_ADAM_V: [t[n + "/Adam_1"] for n in C.CRITIC]}
        self.pw = {0: (float(t["beta1_power"]), float(t["beta2_power"])),
                   1: (float(t["beta1_power_1"]), float(t["beta2_power_1"]))}

    def get_params(self, which):
        return [np.array(x) for x in self.p[which]]

    def set_params(self, which, tensors):
        assert [x.shape for x in tensors] == [x.shape for x in self.p[which]]
        self.p[which] = [np.array(x) for x in tensors]

    def get_adam_powers(self, net):
        return self.pw[net]

    def set_adam_powers(self, net, b1p, b2p):
        self.pw[net] = (b1p, b2p)


def test_saver_save_restore_and_rotation(tmp_path):
    from distributed_ddpg_amd import checkpoint as C
    t = C.read_bundle(REF)
    sess = _FakeSession(t)
    saver = C.Saver(max_to_keep=2)
    d = str(tmp_path / "model_ddpg")
    paths = [saver.save(sess, d + "/model", global_step=g,
                        summary_values=[float(t[v]) for v in C.SUMMARY_VARS]) for g in (99, 120, 130)]
    assert paths[-1].endswith("model-130")
    assert C.latest_checkpoint(d) == os.path.join(d, "model-130")
    assert not os.path.exists(paths[0] + ".index")  # max_to_keep rotated model-99 out
    state = open(os.path.join(d, "checkpoint")).read()
    assert 'model_checkpoint_path: "model-130"' in state and "model-99" not in state
    # written at global_step 120 from the reference's own values: TF's exact bytes
    for ext in (".index", ".data-00000-of-00001"):
        assert open(paths[1] + ext, "rb").read() == open(REF + ext, "rb").read(), ext
    # restore into a session with perturbed state
    sess2 = _FakeSession(t)
    for w in sess2.p:
        sess2.p[w] = [x * 0 + 1 for x in sess2.p[w]]
    sess2.pw = {0: (0.5, 0.5), 1: (0.5, 0.5)}
    back = saver.restore(sess2, C.latest_checkpoint(d))
    for w in sess.p:
        for x, y in zip(sess.p[w], sess2.p[w]):
            np.testing.assert_array_equal(x, y)
    assert sess2.pw == sess.pw
    assert float(back["global_step"]) == 130.0
