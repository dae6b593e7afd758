"""The split sweep's LDS-DMA ring, checked on the built code object and on its schedule (CPU only).

VERDICT r5 item 2: the round-5 4x4x4-MFMA dots experiment faulted (illegal address) and the LDS-DMA
dots gave wrong sums; both issued uncounted inline-asm loads INTO VGPRs (DESIGN §4.2 "The two
round-5 GPU failures").  The product's split sweep (ppls_kernels.hip:496-541) still issues uncounted
inline-asm `global_load_lds_dwordx4` with hand-counted `s_waitcnt vmcnt(k)`; tools/isa_check.py
states why that is safe and what must hold, and these tests check it mechanically:
  * the built kernels: the DMA has no VGPR destination, its M0 write is inside the same asm triple,
    copies come in unbranched runs of exactly CPW, and only split-sweep instantiations use LDS-DMA;
  * the schedule: every instantiation's (SLOTS, RP, CPW) from the built symbols, every row count a
    workgroup can get (0 .. 80, and large ones), both mu modes: no row read before its copies
    landed, no slot refilled before its row was read; a count one row too large is caught;
  * the sources: no other inline asm issues a memory load;
  * the int8 Gram's SYRK ring (ppls_ozaki.hip; the same asm copies): hand wait before
    every barrier, only vmcnt(0 | 2 NC), a drain after the last copy, and its ring restated and
    simulated for every stage count of a split (1 .. 1024) with a negative control.
"""
import os

import pytest

from conftest import ROOT

import sys
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_check as ic   # noqa: E402

LIB = os.path.join(ROOT, "ppls_amd", "libppls_amd.so")


@pytest.fixture(scope="module")
def kernels():
    if not os.path.exists(LIB):
        pytest.fail("ppls_amd/libppls_amd.so not built (python -m ppls_amd.build)")
    fns = ic.functions(ic.disassemble(LIB))
    return {n: ins for n, ins in fns.items() if any(x[1].startswith(ic.DMA) for x in ins)}


def test_only_split_sweep_and_syrk_kernels_use_lds_dma(kernels):
    assert kernels, "no LDS-DMA kernel found: the split sweep should use it"
    other = [n for n in kernels if not ic.split_params(n) and ic.oz_variant(n) is None]
    assert not other, other
    assert any(ic.split_params(n) for n in kernels) and any(ic.oz_variant(n) is not None for n in kernels)


def test_built_split_kernels_dma_form_and_runs(kernels):
    bad = {}
    for n, ins in kernels.items():
        if not ic.split_params(n):
            continue
        pr = ic.check_kernel(ins, ic.split_params(n)[6])
        if pr:
            bad[n[:80]] = pr[:5]
    assert not bad, bad


def test_ring_schedule_every_built_instantiation(kernels):
    shapes = {(p[5], p[3], p[6]) for p in map(ic.split_params, kernels) if p}   # (SLOTS, RP, CPW)
    assert shapes
    for SLOTS, RP, CPW in sorted(shapes):
        for write_mu in (False, True):
            for nrows in list(range(0, 81)) + [127, 128, 129, 1000, 3907, 3908]:
                pr = ic.ring_schedule(nrows, SLOTS, RP, CPW, write_mu)
                assert not pr, (SLOTS, RP, CPW, write_mu, nrows, pr[:3])


def test_ring_schedule_negative_control():
    """A wait count one row (CPW copies) too large must be reported (the model can see a bad k)."""
    for RP in (1, 2):
        for CPW in (2, 4):
            found = any(ic.ring_schedule(n, 4, RP, CPW, False, bias=CPW) for n in range(1, 40))
            assert found, (RP, CPW)


def test_isa_checker_negative_controls():
    """The ISA checker flags a VGPR-destination load, a split asm triple and a short run."""
    good = [(0, "s_mov_b32", "m0, s4", None), (4, "s_nop", "0", None),
            (8, "global_load_lds_dwordx4", "v1, s[2:3]", None)]
    assert not ic.check_kernel(good * 2, 2)
    vdst = [(0, "s_mov_b32", "m0, s4", None), (8, "global_load_dwordx4", "v[4:7], v1, s[2:3]", None)]
    assert ic.check_kernel([(0, "s_mov_b32", "m0, s4", None),
                            (8, "global_load_lds_dwordx4", "v[4:7], v1, s[2:3]", None)] * 2, 2)
    assert not ic.check_kernel(vdst, 2)   # a plain (counted) load is not a DMA copy
    split = [(0, "s_mov_b32", "m0, s4", None), (4, "v_add_u32", "v1, v2, v3", None),
             (8, "global_load_lds_dwordx4", "v1, s[2:3]", None)]
    assert ic.check_kernel(split + good, 2)
    assert ic.check_kernel(good, 2)        # a run of one copy where CPW = 2


def test_no_other_inline_asm_loads():
    assert ic.sources_with_asm_loads() == []


def test_built_syrk_ring_waits(kernels):
    oz = {n: ins for n, ins in kernels.items() if ic.oz_variant(n) is not None}
    assert oz
    bad = {n[:60]: ic.check_oz_kernel(ins)[:5] for n, ins in oz.items() if ic.check_oz_kernel(ins)}
    assert not bad, bad


def test_syrk_ring_schedule_and_negative_control():
    for NC in (4, 8):
        for ns in list(range(1, 41)) + [255, 1023, 1024]:
            pr = ic.ring_schedule_oz(ns, NC)
            assert not pr, (NC, ns, pr[:3])
        # one stage too many in flight at the wait: a read before its copies landed must be caught
        assert any(ic.ring_schedule_oz(ns, NC, bias=NC) for ns in range(2, 20)), NC
    # the checker flags a barrier whose hand wait is missing and a kernel that never drains
    dma = [(0, "s_mov_b32", "m0, s4", None), (4, "s_nop", "0", None), (8, "global_load_lds_dwordx4", "v1, s[2:3]", None)]
    assert ic.check_oz_kernel(dma + [(12, "s_waitcnt", "vmcnt(16)", None), (16, "s_barrier", "", None),
                                     (20, "s_waitcnt", "vmcnt(0)", None)]) == []
    assert ic.check_oz_kernel(dma + [(16, "s_barrier", "", None), (20, "s_waitcnt", "vmcnt(0)", None)])
    assert ic.check_oz_kernel(dma + [(12, "s_waitcnt", "vmcnt(16)", None), (16, "s_barrier", "", None)])


def test_steady_state_wait_is_compiled(kernels):
    """The steady-state wait of the restated ring, vmcnt(AHEAD RP CPW) with AHEAD = SLOTS / RP - 2
    (ppls_kernels.hip:510-512), is an instruction of every built split-sweep instantiation that needs
    one (a count the compiler never sees could otherwise be dropped or merged unnoticed)."""
    import re
    for n, ins in kernels.items():
        p = ic.split_params(n)
        if not p:
            continue
        _, _, _, RP, _, SLOTS, CPW = p
        k = (SLOTS // RP - 2) * RP * CPW
        waits = {int(m) for (_, mn, ops, _) in ins if mn == "s_waitcnt" for m in re.findall(r"vmcnt\((\d+)\)", ops)}
        assert k in waits, (n[:70], k, sorted(waits))
