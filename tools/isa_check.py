"""Static checks of the gfx950 code object inside libddpg_hip.so.

    python tools/isa_check.py [path/to/libddpg_hip.so]

1. Every kernel has zero scratch: .private_segment_fixed_size == 0 and
   .vgpr_spill_count == 0 (from the code object's metadata notes; SGPR spills
   go to VGPR lanes and are allowed).  Exception (EPILOGUE_SPILL_OK): scratch
   outside the MFMA main loop of the 256 x 256-tile GEMM's epilogue forms.
2. No instruction touches a VGPR / AGPR that an in-flight memory read will
   still write ("async-return hazard").  The GEMM kernels read their MFMA
   fragments from LDS with inline-asm ds_read_b128 / ds_read_b64_tr_b16 and
   wait for them with hand-placed s_waitcnt lgkmcnt: the compiler models an
   asm output as written AT the asm statement, so it may spill that register
   or reuse it before the data has returned.  The LDS return then lands on
   whatever the register holds by then.  That is the cause of the aperture
   violation recorded for gemm_h16_kernel<RK,KR,NP=3,128,32>
   (profiles/r2_gemm_ablation/mf16_vs_mf32_with_np3_fault.txt): in its ISA a
   fragment read `ds_read_b128 v[4:7]` is followed, before any lgkmcnt wait,
   by a spill of v[4:7], then by `v_lshl_add_u64 v[4:5], ...` (a staging
   address) and `global_load_lds_dwordx4 v[4:5]` -- the returning fragment
   overwrites the address.

The hazard scan is a dataflow pass over each kernel's control-flow graph.
State: the ordered queues of outstanding LDS reads (lgkmcnt) and vector-memory
ops (vmcnt) with their destination registers.  `s_waitcnt lgkmcnt(N)` keeps
only the newest N LDS ops (LDS returns in order, so an LDS op with more than N
LDS ops issued at or after it has completed -- true whatever SMEM ops are also
counted); `vmcnt(N)` likewise for vector memory; flat ops return out of
order and retire only at vmcnt(0) + lgkmcnt(0); at most 15 / 63 ops are ever
outstanding (the counters' maxima: issue stalls there).  Join = element-wise union
aligned at the newest entry (an over-approximation).  Any later instruction
reading or writing an outstanding destination register is reported.

Build infrastructure (used by __graft_entry__.build() and tests/test_isa.py);
host only, reads the built library, runs nothing on a GPU.
"""
import os
import re
import struct
import subprocess
import sys

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_SO = os.path.join(ROOT, "distributed_ddpg_amd", "libddpg_hip.so")


def code_objects(so_path, arch="gfx950"):
    """Every `arch` code object of the library's .hip_fatbin section: one clang
    offload bundle per translation unit, concatenated (aligned)."""
    out = "/tmp/isa_check_%d.fatbin" % os.getpid()
    copy = out + ".so"  # objcopy writes a copy of its input; discarded
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", ".hip_fatbin=" + out,
                    so_path, copy], check=True, capture_output=True)
    try:
        data = open(out, "rb").read()
    finally:
        for f in (out, copy):
            if os.path.exists(f):
                os.remove(f)
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    if not data.startswith(magic):
        raise ValueError("no clang offload bundle in %s" % so_path)
    cos = []
    start = 0
    while start >= 0:
        (n,) = struct.unpack_from("<Q", data, start + len(magic))
        o = start + len(magic) + 8
        end = start
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, o)
            o += 24
            triple = data[o:o + tlen].decode()
            o += tlen
            end = max(end, start + off + size)
            if triple.endswith(arch) and size:
                cos.append(data[start + off:start + off + size])
        start = data.find(magic, max(end, start + 1))
    if not cos:
        raise ValueError("no %s code object in %s" % (arch, so_path))
    return cos


def code_object(so_path, arch="gfx950"):
    """The first `arch` code object (single-unit libraries)."""
    return code_objects(so_path, arch)[0]


def kernel_resources_all(so_path):
    """kernel_resources merged over every code object of the library."""
    out = {}
    for co in code_objects(so_path):
        out.update(kernel_resources(co))
    return out


def disassemble_all(so_path):
    """disassemble merged over every code object of the library."""
    out = {}
    for co in code_objects(so_path):
        out.update(disassemble(co))
    return out


def _run(tool, co, *args):
    tmp = "/tmp/isa_check_%d.co" % os.getpid()
    with open(tmp, "wb") as f:
        f.write(co)
    try:
        return subprocess.run([os.path.join(LLVM, tool)] + list(args) + [tmp], check=True,
                              capture_output=True, text=True).stdout
    finally:
        os.remove(tmp)


def kernel_resources(co):
    """{kernel symbol: {"scratch", "vgpr_spill", "sgpr_spill", "vgpr"}} from the
    code object's AMDGPU metadata (one YAML map per kernel; .name appears
    after the numeric fields of its map)."""
    notes = _run("llvm-readelf", co, "--notes")
    fields = {".private_segment_fixed_size:": "scratch", ".vgpr_spill_count:": "vgpr_spill",
              ".sgpr_spill_count:": "sgpr_spill", ".vgpr_count:": "vgpr"}
    out, cur = {}, {}
    in_kernels = False
    for line in notes.splitlines():
        s = line.strip()
        if s.startswith("amdhsa.kernels:"):
            in_kernels = True
            continue
        if not in_kernels:
            continue
        if re.match(r"^amdhsa\.", s):
            break
        if s.startswith("- ") and cur:
            # a new list item: flush the previous kernel map
            if "name" in cur:
                out[cur.pop("name")] = cur
            cur = {}
        body = s[2:] if s.startswith("- ") else s
        for f, k in fields.items():
            if body.startswith(f):
                cur[k] = int(body.split(":", 1)[1])
        if body.startswith(".name:") and "name" not in cur:
            cur["name"] = body.split(":", 1)[1].strip()
    if "name" in cur:
        out[cur.pop("name")] = cur
    return out


_INSN = re.compile(r"^\s+([a-z_0-9]+)(.*?)\s*//\s*([0-9A-Fa-f]+):")
_TARGET = re.compile(r"<([^>+]+)\+0x([0-9a-f]+)>")
_REG1 = re.compile(r"\b([va])(\d+)\b")
_REGN = re.compile(r"\b([va])\[(\d+):(\d+)\]")
_HEAD = re.compile(r"^([0-9a-f]+) <([^>]+)>:")


def _regs(text):
    r = set()
    for kind, lo, hi in _REGN.findall(text):
        r.update((kind, i) for i in range(int(lo), int(hi) + 1))
    for kind, i in _REG1.findall(_REGN.sub(" ", text)):
        r.add((kind, int(i)))
    return r


def disassemble(co):
    """{kernel: [(addr, mnemonic, operand text, branch target addr or None)]}"""
    text = _run("llvm-objdump", co, "-d", "--mcpu=gfx950")
    kernels, cur, base = {}, None, 0
    for line in text.splitlines():
        h = _HEAD.match(line)
        if h:
            cur = h.group(2)
            base = int(h.group(1), 16)
            kernels[cur] = []
            continue
        m = _INSN.match(line)
        if not m or cur is None:
            continue
        mn, ops, addr = m.group(1), m.group(2), int(m.group(3), 16)
        t = _TARGET.search(line)
        tgt = base + int(t.group(2), 16) if (t and mn.startswith(("s_branch", "s_cbranch"))) else None
        kernels[cur].append((addr, mn, ops.strip(), tgt))
    return kernels


def _dest_and_kind(mn, ops):
    """(queue, destination registers) of a memory op, or (None, None)."""
    first = ops.split(",")[0] if ops else ""
    if mn.startswith("ds_"):
        has_dst = any(k in mn for k in ("read", "load", "rtn", "permute", "swizzle", "append",
                                        "consume")) and not mn.startswith("ds_write")
        return "lgkm", (_regs(first) if has_dst else set())
    if mn.startswith(("global_", "buffer_", "scratch_", "flat_")):
        # LDS-DMA forms (global_load_lds_*, buffer_load_* ... lds) write LDS,
        # not VGPRs: their first VGPR operand is the address
        lds_dma = "load_lds" in mn or mn.endswith("_lds") or re.search(r"\blds\b", ops) is not None
        loads = ("load" in mn and not lds_dma) or "_rtn" in mn
        if mn.startswith(("global_atomic", "buffer_atomic", "flat_atomic")):
            loads = " glc" in ops or "sc0" in ops
        q = "flat" if mn.startswith("flat_") else "vm"
        return q, (_regs(first) if loads else set())
    return None, None


def _wait(ops):
    w = {}
    for k in ("vmcnt", "lgkmcnt"):
        m = re.search(k + r"\((\d+)\)", ops)
        if m:
            w[k] = int(m.group(1))
    return w


def _join(a, b):
    if a is None:
        return b
    out = []
    for qa, qb in zip(a, b):
        n = max(len(qa), len(qb))
        qa = (frozenset(),) * (n - len(qa)) + qa
        qb = (frozenset(),) * (n - len(qb)) + qb
        out.append(tuple(x | y for x, y in zip(qa, qb)))
    return tuple(out)


def _step(state, mn, ops, report=None):
    lds, vm, fl = state
    if mn == "s_waitcnt":
        w = _wait(ops)
        if "lgkmcnt" in w:
            lds = lds[len(lds) - w["lgkmcnt"]:] if w["lgkmcnt"] < len(lds) else lds
        if "vmcnt" in w:
            vm = vm[len(vm) - w["vmcnt"]:] if w["vmcnt"] < len(vm) else vm
        if w.get("lgkmcnt", 1) == 0 and w.get("vmcnt", 1) == 0:
            fl = ()  # flat ops return out of order: only both counters at 0 retire them
        return (lds, vm, fl)
    q, dst = _dest_and_kind(mn, ops)
    if report is not None:
        used = _regs(ops)
        # a load's own destination may overlap an older load of the same
        # queue: returns are in order, so the older one lands first (WAW is
        # safe; the compiler relies on it)
        own = used - dst if dst else used
        for name, queue, u in (("lgkm", lds, own if q == "lgkm" else used),
                               ("vm", vm, own if q == "vm" else used),
                               ("flat", fl, used)):
            pend = frozenset().union(*queue) if queue else frozenset()
            hit = u & pend
            if hit:
                report(name, sorted(hit))
    if q == "lgkm":
        lds = lds + (frozenset(dst),)
    elif q == "vm":
        vm = vm + (frozenset(dst),)
    elif q == "flat":
        fl = fl + (frozenset(dst),)
    # issue stalls while a counter is at its maximum (gfx9: lgkmcnt 4 bits,
    # vmcnt 6 bits), so older ops have completed
    return (lds[-15:], vm[-63:], fl[-15:])


def store_data_hazards(insns):
    """VMEM stores of more than 8 bytes read their data VGPRs after issue: a
    VALU write of those registers in the next instruction (no wait state
    between) corrupts the stored value.  hipcc inserts the wait for its own
    stores but not after an inline-asm store (the round-4 split-K partial
    stores showed it as run-to-run differences).  [(addr, store, writer)]"""
    out = []
    wide = ("dwordx3", "dwordx4", "_b96", "_b128")
    for i, (a, mn, ops, _) in enumerate(insns[:-1]):
        if not (mn.startswith(("global_store", "buffer_store", "flat_store", "scratch_store")) and
                mn.endswith(wide)):
            continue
        parts = [x.strip() for x in ops.split(",")]
        data = _regs(parts[0] if mn.startswith("buffer_") else (parts[1] if len(parts) > 1 else ""))
        _, nmn, nops, _ = insns[i + 1]
        if nmn.startswith("v_") and nops and _regs(nops.split(",")[0]) & data:
            out.append((a, "%s %s" % (mn, ops), "%s %s" % (nmn, nops)))
    return out


def scan_kernel(insns):
    """Async-return hazards of one kernel: [(addr, insn text, queue, regs)]."""
    if not insns:
        return []
    addrs = [a for a, _, _, _ in insns]
    index = {a: i for i, a in enumerate(addrs)}
    leaders = {0}
    for i, (a, mn, ops, tgt) in enumerate(insns):
        if mn.startswith(("s_branch", "s_cbranch", "s_endpgm", "s_setpc")):
            if i + 1 < len(insns):
                leaders.add(i + 1)
            if tgt is not None and tgt in index:
                leaders.add(index[tgt])
    starts = sorted(leaders)
    blocks = {}
    for j, s in enumerate(starts):
        e = starts[j + 1] if j + 1 < len(starts) else len(insns)
        blocks[s] = (s, e)
    succ = {}
    for s, (b, e) in blocks.items():
        a, mn, ops, tgt = insns[e - 1]
        nxt = []
        if mn.startswith("s_endpgm") or mn.startswith("s_setpc"):
            pass
        elif mn.startswith("s_branch"):
            if tgt in index:
                nxt.append(index[tgt])
        else:
            if mn.startswith("s_cbranch") and tgt in index:
                nxt.append(index[tgt])
            if e < len(insns):
                nxt.append(e)
        succ[s] = nxt
    empty = ((), (), ())
    inst = {0: empty}
    work = [0]
    while work:
        s = work.pop()
        st = inst[s]
        b, e = blocks[s]
        for i in range(b, e):
            st = _step(st, insns[i][1], insns[i][2])
        for n in succ[s]:
            j = _join(inst.get(n), st)
            if j != inst.get(n):
                inst[n] = j
                work.append(n)
    hazards = []
    for s, (b, e) in blocks.items():
        if s not in inst:
            continue
        st = inst[s]
        for i in range(b, e):
            a, mn, ops, _ = insns[i]
            st = _step(st, mn, ops, report=lambda q, r, a=a, mn=mn, ops=ops:
                       hazards.append((a, "%s %s" % (mn, ops), q, r)))
    return hazards


# Kernels allowed scratch OUTSIDE their MFMA main loop: the 256 x 256-tile
# dX GEMM (gemm_h256.h MODE 1) holds 128 accumulator registers per lane into
# its fused epilogue and spills a few epilogue temporaries there.  Allowed
# only if no scratch load lies between the kernel's first and last MFMA (its
# vmcnt wait would drain the LDS-DMA pipeline; an early spill store of an
# epilogue value is harmless), and the hazard scan below -- the correctness
# guard -- still runs on the whole kernel.
EPILOGUE_SPILL_OK = r"gemm_h256_kernelILi\d+ELi\d+ELi[12]E"


def _scratch_in_main_loop(insns):
    mf = [i for i, (_, mn, _, _) in enumerate(insns) if mn.startswith("v_mfma")]
    if not mf:
        return False
    return any(mn.startswith("scratch_load") for _, mn, _, _ in insns[mf[0]:mf[-1] + 1])


def check(so_path=DEFAULT_SO, kernels_like=None, verbose=False):
    """Returns a list of problem strings (empty: the library passes)."""
    problems = []
    res = kernel_resources_all(so_path)
    if not res:
        problems.append("no kernel metadata found")
    dis = disassemble_all(so_path)
    for k, r in sorted(res.items()):
        # (SGPR spills go to VGPR lanes with v_writelane: synchronous, no scratch)
        if r.get("scratch", 0) or r.get("vgpr_spill", 0):
            if re.search(EPILOGUE_SPILL_OK, k) and k in dis and not _scratch_in_main_loop(dis[k]):
                continue
            problems.append("%s: scratch %d B, %d VGPR spills" % (
                k, r.get("scratch", 0), r.get("vgpr_spill", 0)))
    for k, insns in sorted(dis.items()):
        if kernels_like and not re.search(kernels_like, k):
            continue
        for a, st, wr in store_data_hazards(insns)[:5]:
            problems.append("%s +0x%x: %s has its data registers rewritten by %s with no wait state"
                            % (k, a - insns[0][0], st, wr))
        hz = scan_kernel(insns)
        for a, txt, q, r in hz[:5]:
            problems.append("%s +0x%x: %s touches %s registers %s still being written"
                            % (k, a - insns[0][0], txt, q, r[:4]))
        if verbose:
            print("%-100s %6d insns, %d hazards" % (k[:100], len(insns), len(hz)))
    return problems


if __name__ == "__main__":
    pos = [a for a in sys.argv[1:] if not a.startswith("-")]
    so = pos[0] if pos else DEFAULT_SO
    probs = check(so, verbose="-v" in sys.argv)
    for p in probs:
        print(p)
    print("isa_check: %s (%s)" % ("FAIL" if probs else "ok", so))
    sys.exit(1 if probs else 0)
