"""MI355X-native DDPG learner-update hot path (camigord/Distributed_DDPG).

Product path: hand-written gfx950 HIP kernels in libddpg_hip.so behind the
C-ABI of include/ddpg_hip.h, reached through ctypes.  Importing the package
loads the library and fails loudly if it is missing (no CPU fallback).

Reference-interface modules:
  networks       ActorNetwork, CriticNetwork, Session  (reference networks.py)
  replay_buffer  ReplayBuffer                          (reference replay_buffer.py)
  parameters     Parameters                            (reference parameters.py)
  ddpg           --job_name / --task_index CLI         (reference ddpg.py)
  learner        fused learner step + RCCL data parallelism
"""
import os

PACKAGE_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PACKAGE_DIR, "libddpg_hip.so")


def load():
    """Load the HIP library (raises ImportError if it is not built)."""
    from . import _lib
    return _lib
