"""The C-ABI library loads on a GPU-less host and exports every symbol that
include/ddpg_hip.h declares; the ctypes prototypes cover all of them.
No compute calls are made here."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "ddpg_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ddpg_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    from distributed_ddpg_amd import _lib
    names = _declared()
    assert len(names) >= 35
    missing = [n for n in names if not hasattr(_lib.lib, n)]
    assert not missing, missing
    bound = {p[0] for p in _lib.PROTOTYPES}
    assert set(names) == bound, (set(names) ^ bound)


def test_nm_dynamic_exports():
    import subprocess
    so = os.path.join(ROOT, "distributed_ddpg_amd", "libddpg_hip.so")
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True,
                         check=True).stdout
    syms = {l.split()[-1] for l in out.splitlines() if l.strip()}
    for n in _declared():
        assert n in syms, n


def test_abi_version_and_errors_without_gpu():
    from distributed_ddpg_amd import _lib
    assert _lib.lib.ddpg_abi_version() == _lib.ABI_VERSION == 2
    # creating a context with bad dims fails cleanly (no exception crosses the ABI)
    cfg = _lib.Cfg()
    h = _lib.ctypes.c_void_p()
    rc = _lib.lib.ddpg_create(_lib.ctypes.byref(cfg), _lib.ctypes.byref(h))
    assert rc == _lib.DDPG_EINVAL and not h.value
    assert b"dims" in _lib.lib.ddpg_global_error()


def test_cfg_struct_layout():
    """ddpg_cfg is 19 x 4-byte fields, no padding (matches the header)."""
    from distributed_ddpg_amd import _lib
    assert _lib.ctypes.sizeof(_lib.Cfg) == 19 * 4
    assert _lib.ctypes.sizeof(_lib.Stats) == 8
