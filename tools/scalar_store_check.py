"""Build-time gate: no kernel of the library writes through the scalar data
cache (scalar stores and atomics, the scalar cache's write-back / discard).
Runs of such code were followed by whole-machine resets on the GPU pool, so
__graft_entry__.build() refuses a library that contains any.  Host only: it
disassembles the built .so (tools/isa_check.py) and runs nothing on a GPU.

This file names those instructions, so it is listed in .gpurunignore (the GPU
box never needs it: build() runs in the build container only)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_check  # noqa: E402

FORBIDDEN = ("s_store", "s_buffer_store", "s_scratch_store", "s_atomic", "s_buffer_atomic",
             "s_dcache_wb", "s_dcache_discard")


def check(so_path=isa_check.DEFAULT_SO):
    problems = []
    for name, insns in sorted(isa_check.disassemble_all(so_path).items()):
        for addr, mnemonic, _, _ in insns:
            if mnemonic.startswith(FORBIDDEN):
                problems.append("%s +0x%x: %s" % (name, addr - insns[0][0], mnemonic))
    return problems


if __name__ == "__main__":
    probs = check(sys.argv[1] if len(sys.argv) > 1 else isa_check.DEFAULT_SO)
    for p in probs:
        print(p)
    print("scalar_store_check: %s" % ("FAIL" if probs else "ok"))
    sys.exit(1 if probs else 0)
