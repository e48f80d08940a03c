"""Static checks of the built library's gfx950 code object (tools/isa_check.py):
every kernel runs without scratch (no VGPR spills), and no instruction touches
a register that an in-flight LDS / vector-memory read is still going to write.

The second check is what makes the GEMMs' inline-asm fragment reads safe: the
compiler treats an asm output as written at the asm statement, so a spill or
a reuse of that register before the hand-placed lgkmcnt wait lets the LDS
return clobber it.  The round-2 aperture violation of the 16x16x32 NP = 3
twin GEMM was exactly that (profiles/r3/np3_h16_fault_cause.txt); a variant
like it now fails here, at build time, instead of on the GPU.
Host only: reads the .so, runs nothing on a GPU."""
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "distributed_ddpg_amd", "libddpg_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"

pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(LLVM, "llvm-objdump")),
                                reason="ROCm llvm tools absent")


@pytest.fixture(scope="module")
def isa():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_check
    return isa_check


def test_library_has_no_scratch_and_no_async_return_hazards(isa):
    problems = isa.check(SO)
    assert not problems, "\n".join(problems)


def test_every_gemm_and_thin_k_kernel_is_covered(isa):
    res = isa.kernel_resources_all(SO)  # every translation unit's code object
    names = list(res)
    assert any("gemm_h_kernel" in n for n in names)
    assert any("gemm_h16_kernel" in n for n in names)
    assert any("thin_k_kernel" in n for n in names)
    assert any("gemm_h256_kernel" in n for n in names)
    dis = isa.disassemble_all(SO)
    for n in names:
        if re.search(isa.EPILOGUE_SPILL_OK, n):
            # allowed epilogue spills only: no scratch load inside the MFMA main loop
            assert not isa._scratch_in_main_loop(dis[n]), n
        else:
            assert res[n].get("scratch", -1) == 0, n


def test_buffer_load_lds_has_no_vgpr_destination(isa):
    """buffer_load ... lds (LDS-DMA) writes LDS; its VGPR operand is the
    address, so reading / rewriting that VGPR before the DMA lands is fine."""
    insns = [
        (0x0, "buffer_load_dwordx4", "v196, s[0:3], 0 offen lds", None),
        (0x8, "v_add_u32_e32", "v196, 0x40, v196", None),
        (0x10, "s_endpgm", "", None),
    ]
    assert isa.scan_kernel(insns) == []


def test_hazard_scan_catches_async_return_clobber(isa):
    """Synthetic ISA: an LDS read in flight, its destination spilled and then
    reused as an address before the wait -- the pattern of the NP = 3 fault."""
    insns = [
        (0x0, "ds_read_b128", "v[4:7], v0", None),
        (0x8, "scratch_store_dwordx4", "off, v[4:7], off offset:352", None),
        (0x10, "v_lshl_add_u64", "v[4:5], v[244:245], 0, s[8:9]", None),
        (0x18, "global_load_lds_dwordx4", "v[4:5], off", None),
        (0x20, "s_waitcnt", "lgkmcnt(0)", None),
        (0x24, "v_mov_b32_e32", "v4, v5", None),
        (0x28, "s_endpgm", "", None),
    ]
    hz = isa.scan_kernel(insns)
    assert [a for a, *_ in hz] == [0x8, 0x10, 0x18]
    # with the wait first, nothing is reported; an older read is retired by a
    # counted wait that leaves only newer LDS ops outstanding
    ok = [insns[0], (0x4, "ds_read_b128", "v[8:11], v1", None), (0x6, "s_waitcnt", "lgkmcnt(1)", None),
          (0x8, "v_mov_b32_e32", "v4, v5", None), (0xc, "v_mov_b32_e32", "v8, v9", None),
          (0x10, "s_endpgm", "", None)]
    hz = isa.scan_kernel(ok)
    assert [a for a, *_ in hz] == [0xc]


def test_store_data_hazard_detected(isa):
    """A 16-B store whose data registers the next VALU instruction rewrites
    (an inline-asm store hipcc does not pad) is reported; with a wait state
    between, it is not."""
    bad = [(0x0, "global_store_dwordx4", "v[0:1], v[4:7], off sc1", None),
           (0x8, "v_mov_b32_e32", "v5, 0", None), (0xc, "s_endpgm", "", None)]
    assert [a for a, *_ in isa.store_data_hazards(bad)] == [0x0]
    ok = [bad[0], (0x8, "s_nop", "0", None), bad[1], bad[2]]
    assert isa.store_data_hazards(ok) == []
    buf = [(0x0, "buffer_store_dwordx4", "v[4:7], v8, s[0:3], 0 offen sc1", None),
           (0x8, "v_add_f32_e32", "v6, v1, v2", None)]
    assert [a for a, *_ in isa.store_data_hazards(buf)] == [0x0]
