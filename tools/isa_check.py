"""Mechanical checks of the LDS-DMA ring in the BUILT gfx950 code object (no GPU needed).

    python tools/isa_check.py [ppls_amd/libppls_amd.so]

The split sweep (ppls_kernels.hip: ppls_sweep_split_kernel) streams rows HBM -> LDS with
`global_load_lds_dwordx4` issued by inline asm (ppls_device.h: ppls_dma16s), which the compiler does
not count, and waits for them with hand-counted `s_waitcnt vmcnt(k)`: k = the number of copies
issued AFTER the copies the next barrier's reads need.  Vector-memory loads (the DMA and the
compiler's own loads) retire in issue order, so "at most k outstanding" implies that every copy
issued before the newest k has landed -- whatever stores or compiler loads are interleaved (they can
only make a wait stricter).  That argument holds only if

  (1) the DMA has no VGPR destination and its M0 (LDS address) is written in the same asm statement:
      the compiler can neither copy a destination register before the data land (the round-5
      LDS-DMA-dots fault: an uncounted asm load whose destination the register allocator copied) nor
      move code between the M0 write and the copy;
  (2) each row issue is exactly CPW copies in straight-line code (the count k is in units of CPW
      copies per row): the DMA ops form unbranched runs of exactly CPW;
  (3) no kernel other than the split sweep and the int8 Gram's SYRK (ppls_ozaki.hip:
      ppls_oz_syrk_kernel) issues LDS-DMA (no experiment code in the product);
  (4) the k the kernel computes is right: the ring schedule of ppls_kernels.hip:496-541, restated in
      ring_schedule() below, is simulated for every instantiation and every row count of a workgroup
      (in-order retirement, CPW copies per row per DMA wave), checking that every row a workgroup
      reads after a barrier has landed and that no slot is refilled before its row was read;
  (5) no other inline asm in the product issues a memory load (no VGPR-destination asm loads):
      sources_with_asm_loads() scans ppls_amd/csrc.

  (6) the SYRK ring (4 buffers, copies of stage s + 3 issued during stage s, NC = 4 or 8 copies per
      wave per stage): every barrier is preceded by a hand wait vmcnt(2 NC), every vmcnt wait is 0
      or 2 NC, the kernel drains (vmcnt(0)) after its last copy, and ring_schedule_oz() -- the loop
      restated -- reads no stage before its copies landed and refills no buffer before it was read.

tests/test_isa_dma_ring.py runs all six on the product library.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile
from collections import deque

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DMA = ("global_load_lds_", "buffer_load_lds_")  # LDS-DMA mnemonics (gfx950: global_load_lds_dwordx4 ...)


_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def disassemble(lib: str) -> str:
    """llvm-objdump of every gfx950 code object inside a HIP object / shared library (a linked
    library's .hip_fatbin holds one offload bundle per translation unit, back to back)."""
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fb")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fb], check=True)
        blob = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(_MAGIC), blob)]
        out = []
        for k, a in enumerate(starts):
            part, co = os.path.join(d, f"b{k}"), os.path.join(d, f"co{k}")
            with open(part, "wb") as f:
                f.write(blob[a:starts[k + 1] if k + 1 < len(starts) else len(blob)])
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
            out.append(subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co],
                                      capture_output=True, text=True, check=True).stdout)
        return "\n".join(out)


_FUNC = re.compile(r"^([0-9a-f]+) <([^>]+)>:$")
_INS = re.compile(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):(.*)$")
_TGT = re.compile(r"<([^>+]+)\+0x([0-9a-f]+)>")


def functions(dis: str) -> dict:
    """{symbol: [(addr, mnemonic, operands, branch_target_addr or None)]}"""
    out, cur, base = {}, None, 0
    for ln in dis.split("\n"):
        m = _FUNC.match(ln)
        if m:
            base, cur = int(m.group(1), 16), m.group(2)
            out[cur] = []
            continue
        if cur is None:
            continue
        m = _INS.match(ln)
        if not m:
            continue
        mn, ops, addr, tail = m.group(1), m.group(2), int(m.group(3), 16), m.group(4)
        t = _TGT.search(tail)
        tgt = base + int(t.group(2), 16) if (t and mn.startswith(("s_branch", "s_cbranch"))) else None
        out[cur].append((addr, mn, ops, tgt))
    return out


_TARGS = re.compile(r"ppls_sweep_split_kernelILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELb([01])ELi(\d+)ELi(\d+)EE")


def split_params(name: str):
    """(R, NSH, NT, RP, PIPE, SLOTS, CPW) of a split-sweep instantiation from its mangled name."""
    m = _TARGS.search(name)
    return tuple(int(g) for g in m.groups()) if m else None


_OZ = re.compile(r"ppls_oz_syrk_kernelILi(\d+)EE")


def oz_variant(name: str):
    """The SYRK variant V of a ppls_oz_syrk_kernel<V> instantiation, else None."""
    m = _OZ.search(name)
    return int(m.group(1)) if m else None


def dma_form_problems(ins: list) -> list:
    """Check (1) alone: every DMA is the asm triple (s_mov_b32 m0 ; s_nop ; copy vOFF, s[base])."""
    probs = []
    for i, (a, mn, ops, _) in enumerate(ins):
        if not mn.startswith(DMA):
            continue
        fields = [f.strip() for f in ops.replace(" nt", "").split(",")]
        if not (len(fields) == 2 and re.fullmatch(r"v\d+", fields[0]) and re.fullmatch(r"s\[\d+:\d+\]", fields[1])):
            probs.append(f"{a:x}: DMA operands not (vOFF, s[base]): {mn} {ops}")
        j = i - 1
        while j >= 0 and ins[j][1] == "s_nop":
            j -= 1
        if j < 0 or ins[j][1] != "s_mov_b32" or not ins[j][2].startswith("m0,"):
            probs.append(f"{a:x}: DMA not directly preceded by its s_mov_b32 m0")
    return probs


_VMC = re.compile(r"vmcnt\((\d+)\)")


def check_oz_kernel(ins: list) -> list:
    """Check (6) on the built SYRK: hand waits before barriers, wait counts, the final drain."""
    probs = dma_form_problems(ins)
    ks = {int(m.group(1)) for (_, mn, ops, _) in ins if mn == "s_waitcnt" for m in [_VMC.search(ops)] if m}
    if not ks <= {0, 8, 16}:
        probs.append(f"vmcnt waits {sorted(ks)}: only 0 and 2 NC (8 on the diagonal, 16 off it) are scheduled")
    for i, (a, mn, _, _) in enumerate(ins):
        if mn != "s_barrier":
            continue
        k, j = None, i - 1
        while j >= 0 and not ins[j][1].startswith(DMA) and ins[j][1] not in ("s_barrier",):
            if ins[j][1] == "s_waitcnt":
                m = _VMC.search(ins[j][2])
                if m:
                    k = int(m.group(1))
                    break
            j -= 1
        if k not in (8, 16):
            probs.append(f"{a:x}: barrier without its hand wait vmcnt(8 | 16) after the last copy (found {k})")
    last_dma = max((n for n, x in enumerate(ins) if x[1].startswith(DMA)), default=None)
    if last_dma is not None:
        tail = ins[last_dma + 1:]
        drained = any(x[1] == "s_waitcnt" and _VMC.search(x[2]) and int(_VMC.search(x[2]).group(1)) == 0 for x in tail)
        if not drained:
            probs.append("no vmcnt(0) after the last copy: copies could land after the workgroup's LDS is gone")
    return probs


def ring_schedule_oz(nstages: int, NC: int, bias: int = 0) -> list:
    """Restatement of ppls_oz_syrk_kernel's ring (V = 512; ppls_ozaki.hip, `run`): 4 buffers, the
    prologue copies stages 0..2 (clamped to the last stage), step s waits vmcnt <= 2 NC, barriers,
    reads stage s from buffer s % 4 and copies stage min(s + 3, last) into buffer (s + 3) % 4; the
    tail drains.  One wave, in-order retirement.  bias is added to the wait (negative control)."""
    q = deque()                 # outstanding copies: (buffer, stage)
    buf = {}                    # buffer -> stage it holds or is receiving
    read = set()
    probs = []
    last = lambda s: min(s, nstages - 1)

    def issue(b, st):
        old = buf.get(b)
        if old is not None and old not in read and old != st:
            probs.append(f"stage {st} refills buffer {b} before stage {old} was read")
        buf[b] = st
        q.extend([(b, st)] * NC)

    if nstages <= 0:
        return probs
    for k in range(3):
        issue(k, last(k))
    for s in range(nstages):
        while len(q) > 2 * NC + bias:
            q.popleft()
        # barrier; every wave's copies of stage s landed (each waited for its own)
        if any(b == s % 4 for (b, _) in q):
            probs.append(f"stage {s} read while a copy into its buffer is in flight")
        if buf.get(s % 4) != s:
            probs.append(f"stage {s}'s buffer holds stage {buf.get(s % 4)}")
        read.add(s)
        issue((s + 3) % 4, last(s + 3))
    q.clear()
    return probs


def check_kernel(ins: list, cpw: int) -> list:
    """Problems of checks (1) and (2) in one kernel's instruction list (empty: clean)."""
    probs = []
    targets = {t for (_, _, _, t) in ins if t is not None}
    run, run_start = 0, None

    def end_run():
        nonlocal run
        if run and run != cpw:
            probs.append(f"{run_start:x}: a run of {run} DMA copies, not CPW = {cpw}")
        run = 0

    for i, (a, mn, ops, _) in enumerate(ins):
        if a in targets:          # a label: control can enter here, so a run cannot continue across it
            end_run()
        if mn.startswith(DMA):
            # (1) the asm triple: s_mov_b32 m0, sX ; s_nop 0 ; global_load_lds_dwordx4 vOFF, s[..] [nt]
            fields = [f.strip() for f in ops.replace(" nt", "").split(",")]
            if not (len(fields) == 2 and re.fullmatch(r"v\d+", fields[0]) and re.fullmatch(r"s\[\d+:\d+\]", fields[1])):
                probs.append(f"{a:x}: DMA operands not (vOFF, s[base]): a VGPR destination or another form: {mn} {ops}")
            j = i - 1
            while j >= 0 and ins[j][1] == "s_nop":
                j -= 1
            if j < 0 or ins[j][1] != "s_mov_b32" or not ins[j][2].startswith("m0,"):
                probs.append(f"{a:x}: DMA not directly preceded by its s_mov_b32 m0 (code moved into the asm triple)")
            if run == 0:
                run_start = a
            run += 1
            continue
        # (2) a run ends at any branch, barrier, wait or other memory instruction: it must hold
        # exactly CPW copies (address arithmetic in between is fine)
        if mn.startswith(("s_branch", "s_cbranch", "s_barrier", "s_waitcnt", "s_endpgm", "ds_", "global_",
                          "buffer_", "flat_", "scratch_")):
            end_run()
    end_run()
    return probs


def ring_schedule(nrows: int, SLOTS: int, RP: int, CPW: int, write_mu: bool, bias: int = 0) -> list:
    """Restatement of ppls_sweep_split_kernel's ring (ppls_kernels.hip:496-541) for ONE DMA wave
    (CPW copies per row; a wave that issues none waits on nothing and meets the others at the
    barriers).  Simulates in-order retirement; returns the violations found.  bias: added to every
    non-zero wait count (a negative control: a count one row too large must be caught)."""
    AHEAD = SLOTS // RP - 2
    ngroups = (nrows + RP - 1) // RP
    q = deque()                 # outstanding copies: the row each one fills
    slot_row = {}               # slot -> row whose data it holds or is receiving
    read_done = set()           # rows consumed (loaded into registers by every wave)
    probs = []

    def issue_row(i):
        s = i % SLOTS
        old = slot_row.get(s)
        if old is not None and old not in read_done:
            probs.append(f"row {i} refills slot {s} before row {old} was read")
        slot_row[s] = i
        q.extend([i] * CPW)

    def wait(k):
        k = k + bias if k > 0 else k
        while len(q) > k:
            q.popleft()

    def read_group(grp):        # after a barrier: rows of group grp are read from their slots
        for j in range(RP):
            row = min(grp * RP + j, nrows - 1)
            if row in q:
                probs.append(f"row {row} read before its copies landed")
            if slot_row.get(row % SLOTS) != row:
                probs.append(f"row {row}'s slot holds row {slot_row.get(row % SLOTS)}")
            read_done.add(row)

    if ngroups > 0:
        npro = min(SLOTS, nrows)
        for i in range(npro):
            issue_row(i)
        wait(0 if write_mu else (npro - min(RP, nrows)) * CPW)
        read_group(0)                                   # load_x(0) after the prologue barrier
        for gg in range(ngroups):
            if write_mu:
                wait(0)
            elif (gg + 2 + AHEAD) * RP <= nrows and gg >= 1:
                wait(AHEAD * RP * CPW)
            else:
                last_issued = min((gg - 1) * RP + SLOTS + RP - 1 if gg >= 1 else SLOTS - 1, nrows - 1)
                wait(max(0, last_issued - ((gg + 2) * RP - 1)) * CPW)
            # barrier: group gg's rows were read (into xc) before it, by every wave
            if gg * RP + SLOTS < nrows:
                g2 = gg + SLOTS // RP
                for j in range(RP):
                    if g2 * RP + j < nrows:
                        issue_row(g2 * RP + j)
            if gg + 1 < ngroups:
                read_group(gg + 1)
    return probs


def sources_with_asm_loads(csrc: str = os.path.join(ROOT, "ppls_amd", "csrc")) -> list:
    """(file, line, text) of every inline-asm statement in the product sources that names a memory
    load, other than the two DMA helpers of ppls_device.h (check (5))."""
    out = []
    for f in sorted(os.listdir(csrc)):
        if not f.endswith((".hip", ".h", ".cpp")):
            continue
        txt = open(os.path.join(csrc, f)).read()
        for m in re.finditer(r"asm\s*(volatile)?\s*\(\s*\"([^;]*?)\"\s*:", txt):
            body = m.group(2)
            if re.search(r"(global|buffer|flat|scratch)_load|s_load|s_buffer_load|ds_read", body):
                line = txt.count("\n", 0, m.start()) + 1
                helper = "global_load_lds_dwordx4 %1, %2" in body
                if not helper:
                    out.append((f, line, body[:80]))
    return out


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "ppls_amd", "libppls_amd.so")
    fns = functions(disassemble(lib))
    total = 0
    for name, ins in sorted(fns.items()):
        n_dma = sum(1 for x in ins if x[1].startswith(DMA))
        if not n_dma:
            continue
        pr = split_params(name)
        if pr:
            probs = check_kernel(ins, pr[6])
        elif oz_variant(name) is not None:
            probs = check_oz_kernel(ins)
        else:
            probs = [f"LDS-DMA in a kernel that is not the split sweep or the SYRK: {name}"]
        total += len(probs)
        print(f"{name[:90]}: {n_dma} DMA ops, {len(ins)} instructions, {len(probs)} problems")
        for p in probs[:10]:
            print("   ", p)
    sys.exit(1 if total else 0)


if __name__ == "__main__":
    main()
