"""Read extents of the panel sweep's MFMA dots against its allocations (CPU only).

The round-5 4x4x4-MFMA dots experiment died of an illegal address at r = 1 in fp64 storage (DESIGN
§4.2).  Its source was never committed, so the faulting access cannot be replayed; its B operand
loads (three times the product's) are the prime suspect, and the one thing they shared with the
product is the layout they read: X / Y rows (ld_of) with 64 doubles of zeroed slack after the last
row, and Z = [Xw | Yc | mu_T | mu_U] followed by the transposed Wt, Ct with NO slack after Ct
(ppls_panel_z_len).  This test restates the product kernel's addressing (ppls_kernels.hip:
ppls_panel_mfmadots_kernel, load_tile / step) and checks, over a grid of shapes, that its largest
element index stays inside each allocation (ppls_capi.cpp: ld_of, set_data's slack;
ppls_kernels.hip: ppls_panel_z_len, launch_panel_t's Wt / Ct placement).
"""
import itertools


def ld_of(p, f32, pad=1):   # ppls_capi.cpp:215
    es = 4 if f32 else 8
    b = p * es
    if not pad or b < 1024 or (not f32 and p <= 2048):
        return (p + 3) & ~3 if f32 else (p + 1) & ~1
    al = 4096 if b >= 16384 else 128
    return ((b + al - 1) // al * al) // es


def z_len(n, ldx, ldy, r):   # ppls_panel_z_len (doubles)
    return max(n, 1) * 4 * r + (((ldx + 31) & ~31) + ((ldy + 31) & ~31)) * 16


def dots_max_reads(n, p, ld, f32, r, ldx, ldy, is_y):
    """(largest element index of X / Y read, largest double index of Z read through Wt / Ct)."""
    ES = 4 if f32 else 8
    KT = 128 // ES
    KQ = KT // 4
    ntc = (p + KT - 1) // KT
    # load_tile: src[u] = M + rr ld + lchunk (16 / ES) (rr <= n - 1), + c KT for c <= ntc - 1, a 16-B read
    x_max = (n - 1) * ld + 7 * (16 // ES) + (ntc - 1) * KT + 16 // ES - 1
    # step: wb0 = Wm + kq KQ 16 + 2 i16; wb = wb0 + tc KT 16; double2 at wb + s2 16, s2 < KQ (even)
    w_max = 3 * KQ * 16 + 2 * 15 + (ntc - 1) * KT * 16 + (KQ - 2) * 16 + 1
    ldxp = (ldx + 31) & ~31
    base = max(n, 1) * 4 * r + (ldxp * 16 if is_y else 0)   # Wt after Z's rows, Ct after Wt
    return x_max, base + w_max


def test_panel_dots_reads_stay_inside_their_allocations():
    checked = 0
    for f32, p, q, n, r in itertools.product((0, 1), (1, 2, 3, 15, 16, 17, 30, 31, 33, 127, 255, 500, 1023, 2049,
                                                      4097, 10000), (1, 5, 20, 64, 500), (1, 2, 150, 4097), (1, 10)):
        if p < r or q < r:
            continue
        ldx, ldy = ld_of(p, f32), ld_of(q, f32)
        es = 4 if f32 else 8
        for is_y, pc, ld in ((0, p, ldx), (1, q, ldy)):
            x_max, z_max = dots_max_reads(n, pc, ld, f32, r, ldx, ldy, is_y)
            # set_data: (n ld es + 7) / 8 + 64 doubles, i.e. this many elements of the storage type
            alloc_elems = ((max(n, 1) * ld * es + 7) // 8 + 64) * 8 // es
            assert x_max < alloc_elems, (f32, p, q, n, r, is_y, x_max, alloc_elems)
            assert z_max < z_len(n, ldx, ldy, r), (f32, p, q, n, r, is_y, z_max, z_len(n, ldx, ldy, r))
            checked += 1
    assert checked > 500
