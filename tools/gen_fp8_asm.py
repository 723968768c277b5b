#!/usr/bin/env python3
"""Generate the hand-scheduled main loop of the per-tensor fp8 GEMM (csrc/kernels/fp8_gemm_asm.hip).

Writes `accelerate_hpc_test_amd/csrc/kernels/fp8_asm_loop.inc`: one C string macro, `FP8ASM_MAIN_LOOP`, that is
the body of a single `asm volatile` statement in `fp8_gemm_asm_kernel`. The output file is checked in; rerun this
script after editing the schedule below (`python tools/gen_fp8_asm.py`).

Why a generated asm loop (profiles/r4_gemm_fp8.md, "16x16x128 in HIP is register-allocation bound"): the 256x256
tile at 16x16x128 keeps 8x8 accumulator blocks = 256 fp32 per lane. hipcc splits them between VGPRs and AGPRs and
shuffles them with v_accvgpr_mov inside the K-loop; here the accumulators live in a[0:255] for the whole loop and
the 16 operand fragments of one K-tile (A 0..7, B 0..7, 8 VGPRs each) in v[128:255], so the loop is nothing but
MFMAs, ds_reads, LDS-DMA issues and a few scalar ops.

Schedule (one K-tile = 128 fp8 bytes of K = one MFMA K; 4 waves, wave (wm, wn) owns a 128x128 output block;
fragment i of a wave = rows 8r + i, r = 0..15, so each lane ends up with 8 consecutive output columns per row):

  registers at the top of tile t:  A0..A3 and B0..B3 of tile t (read during tile t-1)
  phase 1  MFMA A0-3 x B0-3  | ds_read B4-7 of t | lgkmcnt(0) + barrier (every wave done with B of t)
                             | DMA 5/8 of B(t+2) into the same buffer | ds_read A4-7 of t
  phase 2  MFMA A0-3 x B4-7  | DMA 3/8 of B(t+2) | lgkmcnt(0) + barrier (every wave done with A of t)
                             | DMA 2/8 of A(t+2)
  phase 3  MFMA A4-7 x B0-3  | DMA 5/8 of A(t+2) | vmcnt(15) + barrier (tile t+1 landed for every wave)
  phase 4  MFMA A4-7 x B4-7  | ds_read A0-3, B0-3 of t+1 from the other buffer | DMA 1/8 of A(t+2) | lgkmcnt(0)

Two LDS buffers (one K-tile of A and B each, 2 x 2 x 33 KiB): a tile's buffer is refilled with tile t+2 as soon as
every wave holds tile t in registers, so two tiles are in flight with only two buffers. LDS image of one operand:
32 chunks of 8 rows x 128 B (one wave-wide buffer_load_dwordx4 ... lds each) at a 1056-B stride (32 B pad); the
fragment reads (lane (r, g): row 8r + i, bytes 16g and 64 + 16g) are then conflict-free for all four ds_read_b128
lane groups.

The tail runs the same body twice without DMA (tile nk-2 waits vmcnt(0) for nk-1; tile nk-1 reads nothing).

MN-major A (`BF16AMN_*`, bf16 only): A is stored [K][M] (the M index contiguous: dy of a weight gradient, W of a
dgrad computed as its transpose). One K-tile of A is then 64 k-rows x 512 B (the tile's 256 columns); a DMA chunk
holds two k-rows (1 KiB, same 1056-B chunk stride as the K-major image). Chunk n = q | G'<<2 | (k>>4)<<3 holds rows
k with k&3 = q, bit 3 = G' and bit 2 = the row inside the chunk, so the eight rows one half-wave of a transposed read
touches sit in eight consecutive chunks: at a 1056-B stride they start 32 B apart modulo 256 and the 32 lanes' 8-B
pieces cover all 64 banks once. Fragments come out of LDS through `ds_read_b64_tr_b16` (4 per fragment instead of 2
`ds_read_b128`): lane 4q + p of a 16-lane group g supplies row 8g + 4s + q (+32 for the second MFMA of the K-tile),
columns 4p..4p+3 of its block; block i = 16 consecutive output rows 16i..16i+15 of the wave's 128. One address VGPR
serves all 32 reads of a K-tile (immediate offsets 16896 h + 512 s + 32 i).

MN-major A and B (`BF16ABMN_*`): B takes the same image and transposed reads (block j = 16 consecutive output columns);
the kernel then stores C^T (the accumulator's registers run along A's rows), so the 16-column blocks never have to be
re-packed for 16-byte stores. B's K-tile step is s69; its soffsets reuse s48..s54 (the host passes 8 rows x ldb).
"""

from __future__ import annotations

import os
import sys

# register map (must match fp8_gemm_asm.hip)
A_BASE = 128  # A fragment i = v[128 + 8i : 135 + 8i]
B_BASE = 192  # B fragment j = v[192 + 8j : 199 + 8j]
SRD_A = 40    # s[40:43]
SRD_B = 44    # s[44:47]
SOFF = 48     # s48..s54 = j * 32 * K, j = 1..7
M0_A = 56     # LDS-DMA destination of this wave's first A chunk in the current buffer
M0_B = 57
M0_X = 58     # xor toggling the A destination between buffer 0 and 1
M0_XB = 55    # the same for B (an xor mask toggles only the base it was computed from)
CNT = 59      # main-loop trips left
M0_KEEP = 60  # caller's m0
CHUNK_STEP = 4 * 1056  # m0 advance per DMA instruction (4 waves x one 1056-B chunk)
SOFF_A = 61   # MN-major A: s61..s67 = j * 8 rows * lda, j = 1..7
ADV_A = 68    # MN-major A: bytes between K-tiles (64 rows * lda)
ADV_B = 69    # MN-major B: bytes between K-tiles (64 rows * ldb); its soffsets reuse s48..s54 (= j * 8 rows * ldb)


def A(i):
    return f"v[{A_BASE + 8 * i}:{A_BASE + 8 * i + 7}]"


def B(j):
    return f"v[{B_BASE + 8 * j}:{B_BASE + 8 * j + 7}]"


def acc(i, j):
    b = (i * 8 + j) * 4
    return f"a[{b}:{b + 3}]"


def mfma(i, j):
    return f"v_mfma_f32_16x16x128_f8f6f4 {acc(i, j)}, {A(i)}, {B(j)}, {acc(i, j)} cbsz:%c[fa] blgp:%c[fb]"


def mfma_bf16(i, j, half):
    """bf16: a 128-byte K-tile is 64 elements = two v_mfma_f32_16x16x32_bf16 per accumulator block; lane (r, g)'s
    fragment registers 0-3 hold elements 8g..8g+7 of the first 32 (bytes 16g..), registers 4-7 those of the second."""
    a0, b0 = A_BASE + 8 * i + 4 * half, B_BASE + 8 * j + 4 * half
    return f"v_mfma_f32_16x16x32_bf16 {acc(i, j)}, v[{a0}:{a0 + 3}], v[{b0}:{b0 + 3}], {acc(i, j)}"


def ds_frag(dst_base, f, addr):
    """two ds_read_b128 of fragment slot f (0..7) into v[dst : dst+7] from lane address `addr`"""
    d = dst_base + 8 * f
    return [f"ds_read_b128 v[{d}:{d + 3}], {addr} offset:{128 * f}",
            f"ds_read_b128 v[{d + 4}:{d + 7}], {addr} offset:{128 * f + 64}"]


def ds_frag_tr(f, addr, base=A_BASE):
    """MN-major fragment f: four ds_read_b64_tr_b16 (MFMA half h, k sub-block s) into v[d + 4h + 2s : +1]"""
    d = base + 8 * f
    return [f"ds_read_b64_tr_b16 v[{d + 4 * h + 2 * s}:{d + 4 * h + 2 * s + 1}], {addr} offset:{16896 * h + 512 * s + 32 * f}"
            for h in range(2) for s in range(2)]


# fp8 MN-major image (`mn8`): a 1 KiB chunk = 4 k-rows x 256 B, chunk stride 1040 B (16 B pad: rows in consecutive
# chunks start 16 B apart modulo 256). Row k of a K-tile sits in chunk (k & 7) | ((k >> 4) & 1) << 3 | (k >> 6) << 4 at
# row ((k >> 3) & 1) | ((k >> 5) & 1) << 1, so the 16 k-rows one half-wave of a ds_read_b64_tr_b8 touches (8 rows of
# two 16-lane groups) fall in 16 consecutive chunks and their 16-B pieces cover the 64 banks once. Fragment registers
# 2s, 2s + 1 hold the k-run s of lane group g: k = 16 g + (0, 8, 64, 72)[s] .. +7 (the 16x16x128 f8 operand's bytes
# 16 g .. 16 g + 15 and 64 + 16 g .. 64 + 16 g + 15), read at immediate offsets (0, 256, 16640, 16896)[s] + 16 i.
MN8_CHUNK = 1040
MN8_RUN_OFF = (0, 256, 16 * MN8_CHUNK, 16 * MN8_CHUNK + 256)
MN8_ROW_OFF = (4, 16, 20, 64, 68, 80, 84)  # k-row of DMA instruction j (j = 1..7) of wave 0, lane 0: soffset = row * ld


def ds_frag_tr8(f, addr, base=A_BASE):
    """fp8 MN-major fragment f: four ds_read_b64_tr_b8 (k-run s) into v[d + 2s : +1]"""
    d = base + 8 * f
    return [f"ds_read_b64_tr_b8 v[{d + 2 * s}:{d + 2 * s + 1}], {addr} offset:{MN8_RUN_OFF[s] + 16 * f}" for s in range(4)]


def a_frag(f, amn, mn8=False):
    if amn:
        return ds_frag_tr8(f, "%[va]") if mn8 else ds_frag_tr(f, "%[va]")
    return ds_frag(A_BASE, f, "%[va]")


def b_frag(f, bmn, mn8=False):
    if bmn:
        return ds_frag_tr8(f, "%[vb]", B_BASE) if mn8 else ds_frag_tr(f, "%[vb]", B_BASE)
    return ds_frag(B_BASE, f, "%[vb]")


PROBE_LOADS = [None]
SPREAD = [False]  # bf16 body in the spread issue order (BF16ASM_SPREAD_MAIN_LOOP)  # "regload" / "regstage": the DMA slots issue register loads (+ LDS writes) instead (timing probe)


def dma(op, n, amn=False, mn8=False):
    """n-th (0..7) DMA instruction of operand op ('A'|'B'); m0 must hold this instruction's destination. `amn`: this
    operand is MN-major; `mn8`: in the fp8 MN image (1040-B chunks)."""
    srd = SRD_A if op == "A" else SRD_B
    if PROBE_LOADS[0] is not None:
        so = "0" if n == 0 else f"s{SOFF + n - 1}"
        out = [f"buffer_load_dwordx4 v[252:255], %[voff], s[{srd}:{srd + 3}], {so} offen"]
        if PROBE_LOADS[0] == "regstage":
            out.append(f"ds_write_b128 %[va], v[248:251] offset:{1024 * n}")
        return out
    step = 4 * MN8_CHUNK if (amn and mn8) else CHUNK_STEP
    if op == "A" and amn:
        so = "0" if n == 0 else f"s{SOFF_A + n - 1}"
        out = [f"buffer_load_dwordx4 %[voffa], s[{srd}:{srd + 3}], {so} offen lds"]
    else:
        so = "0" if n == 0 else f"s{SOFF + n - 1}"
        out = [f"buffer_load_dwordx4 %[voff], s[{srd}:{srd + 3}], {so} offen lds"]
    if n < 7:
        out.append(f"s_add_u32 m0, m0, {step}")
    return out


def advance_srd(op, amn=False):
    """`amn`: this operand is MN-major (its K-tile step is a whole row block, held in an SGPR)"""
    srd = SRD_A if op == "A" else SRD_B
    step = (f"s{ADV_A}" if op == "A" else f"s{ADV_B}") if amn else "128"
    return [f"s_add_u32 s{srd}, s{srd}, {step}", f"s_addc_u32 s{srd + 1}, s{srd + 1}, 0"]


def body(dma_on: bool, wait_next: bool, read_next: bool, bf16: bool = False, amn: bool = False, bmn: bool = False,
         reads_on: bool = True, mn8: bool = False):
    """one K-tile; returns a list of instruction lines. Extra work is attached after MFMA #k via `slots[k]`. bf16:
    each accumulator block takes two MFMAs; in every run of four blocks (same A fragment) the four first halves are
    issued, each followed by its slot's work, then the four second halves (4 MFMAs between dependent ones)."""
    slots = {k: [] for k in range(64)}
    order = ([(i, j) for i in range(4) for j in range(4)] + [(i, j) for i in range(4) for j in range(4, 8)]
             + [(i, j) for i in range(4, 8) for j in range(4)] + [(i, j) for i in range(4, 8) for j in range(4, 8)])
    # phase 1: B4-7 of t, then (after the barrier) B DMA 0..4 and A4-7 of t
    for f in range(4 if reads_on else 0):
        slots[f] += b_frag(4 + f, bmn, mn8)
    if dma_on:
        slots[5] += [f"s_mov_b32 m0, s{M0_B}"]
    slots[5] += ["s_waitcnt lgkmcnt(0)"]
    slots[6] += ["s_barrier"]
    if dma_on:
        for n in range(5):
            slots[8 + n] += dma("B", n, bmn, mn8)
    for f in range(3 if reads_on else 0):
        slots[13 + f] += a_frag(4 + f, amn, mn8)
    # phase 2
    if reads_on:
        slots[16] += a_frag(7, amn, mn8)
    slots[20] += ["s_waitcnt lgkmcnt(0)"]
    slots[21] += ["s_barrier"]
    if dma_on:
        for n in range(5, 8):
            slots[22 + n - 5] += dma("B", n, bmn, mn8)
        slots[24] += [f"s_mov_b32 m0, s{M0_A}"]
        slots[28] += advance_srd("B", bmn)  # the SRD bases always point at the next K-tile to load
        for n in range(2):
            slots[25 + n] += dma("A", n, amn, mn8)
        # phase 3
        for n in range(2, 7):
            slots[38 + n - 2] += dma("A", n, amn, mn8)
    if wait_next:
        slots[45] += ["s_waitcnt vmcnt(15)" if dma_on else "s_waitcnt vmcnt(0)"]
        slots[46] += ["s_barrier"]
    # phase 4: lo fragments of t+1 from the other buffer
    if read_next:
        slots[47] += ["v_xor_b32 %[va], %[vax], %[va]", "v_xor_b32 %[vb], %[vbx], %[vb]"]
        for f in range(4 if reads_on else 0):
            slots[48 + f] += b_frag(f, bmn, mn8)
        for f in range(4 if reads_on else 0):
            slots[52 + f + (1 if f >= 1 else 0)] += a_frag(f, amn, mn8)
    if dma_on:
        slots[53] += dma("A", 7, amn, mn8)
        slots[55] += advance_srd("A", amn)
        slots[57] += [f"s_xor_b32 s{M0_A}, s{M0_A}, s{M0_X}", f"s_xor_b32 s{M0_B}, s{M0_B}, s{M0_XB}"]
    if read_next:
        slots[61] += ["s_waitcnt lgkmcnt(0)"]
    lines = []
    if not bf16 and SPREAD[0]:
        # fp8: the same evenly spread single operations over each quadrant's 16 MFMA gaps
        for q in range(4):
            ops = []
            for k in range(16 * q, 16 * q + 16):
                cur = []
                for ins in slots[k]:
                    cur.append(ins)
                    if not ins.startswith(("s_mov_b32 m0", "s_add_u32 s", "s_addc_u32", "s_xor_b32", "v_xor_b32")):
                        ops.append(cur)
                        cur = []
                if cur:
                    ops.append(cur)
            pos = {}
            for n, op in enumerate(ops):
                pos.setdefault(min(15, (n * 16) // max(1, len(ops))), []).extend(op)
            for g, (i, j) in enumerate(order[16 * q : 16 * q + 16]):
                lines.append(mfma(i, j))
                lines += pos.get(g, [])
        return lines
    if not bf16:
        for k, (i, j) in enumerate(order):
            lines.append(mfma(i, j))
            lines += slots[k]
        return lines
    if SPREAD[0]:
        # bf16, hipBLASLt-like issue order: per quadrant (16 blocks) the 16 first-half MFMAs, then the 16 second halves
        # (a block's two MFMAs 16 apart); the quadrant's slot work is cut into single memory / wait / barrier
        # operations (each with the scalar ops that feed it) and laid out evenly over its 32 MFMA gaps, in order.
        # +2.3-3.6 % over the run-of-four order on the 4-wave kernel (profiles/r6_gemm_diagnostics.md).
        for q in range(4):
            ops = []
            for k in range(16 * q, 16 * q + 16):
                cur = []
                for ins in slots[k]:
                    cur.append(ins)
                    if not ins.startswith(("s_mov_b32 m0", "s_add_u32 s", "s_addc_u32", "s_xor_b32", "v_xor_b32")):
                        ops.append(cur)
                        cur = []
                if cur:
                    ops.append(cur)
            blocks = order[16 * q : 16 * q + 16]
            mf = [mfma_bf16(i, j, 0) for (i, j) in blocks] + [mfma_bf16(i, j, 1) for (i, j) in blocks]
            pos = {}
            for n, op in enumerate(ops):
                pos.setdefault(min(31, (n * 32) // max(1, len(ops))), []).extend(op)
            for g in range(32):
                lines.append(mf[g])
                lines += pos.get(g, [])
        return lines
    for c in range(0, 64, 4):
        for k in range(c, c + 4):
            lines.append(mfma_bf16(*order[k], 0))
            lines += slots[k]
        for k in range(c, c + 4):
            lines.append(mfma_bf16(*order[k], 1))
    return lines


def frag_half(base, f, half, addr):
    """one ds_read_b128: half `half` (K elements 32 half ..) of fragment f into v[base + 8f + 4 half : +3]"""
    d = base + 8 * f + 4 * half
    return f"ds_read_b128 v[{d}:{d + 3}], {addr} offset:{128 * f + 64 * half}"


def body_kh(dma_on: bool, wait_next: bool, read_next: bool):
    """bf16 K-tile in K-half order (the issue order of hipBLASLt's MT256x256x64 kernel): the 64 first-half MFMAs of
    all 8 x 8 blocks, then the 64 second halves. Stage H0 reads this tile's second halves (16 ds_read_b128 into the
    registers H1 of the previous tile left), then every wave holds the tile: lgkmcnt(0) + barrier, and the 16 DMAs of
    tile t+2 into this buffer start, one per 4 MFMAs, running into H1. H1 waits for tile t+1 (vmcnt + barrier) and reads
    its first halves into the registers H0 just released."""
    gaps = {g: [] for g in range(128)}
    reads_h1 = [frag_half(B_BASE, f, 1, "%[vb]") for f in range(8)] + [frag_half(A_BASE, f, 1, "%[va]") for f in range(8)]
    for n, r in enumerate(reads_h1):
        gaps[2 * n] += [r]
    gaps[32] += ["s_waitcnt lgkmcnt(0)"]
    gaps[33] += ["s_barrier"]  # every wave holds all of tile t: tile t+2 may overwrite its buffer
    nd = 0
    if dma_on:
        gaps[34] += [f"s_mov_b32 m0, s{M0_B}"]
        g = 35
        for op in ("B", "A"):
            for n in range(8):
                gaps[g] += dma(op, n)
                g += 4
                nd += 1
                if op == "B" and n == 7:
                    gaps[g - 2] += advance_srd("B") + [f"s_mov_b32 m0, s{M0_A}"]
        gaps[g - 2] += advance_srd("A") + [f"s_xor_b32 s{M0_A}, s{M0_A}, s{M0_X}", f"s_xor_b32 s{M0_B}, s{M0_B}, s{M0_XB}"]
    if wait_next:
        # DMAs of this iteration issued before gap 66: (66 - 35) // 4 + 1 = 8
        issued = sum(1 for gg in range(35, 66) for x in gaps[gg] if x.startswith("buffer_load"))
        gaps[66] += [f"s_waitcnt vmcnt({issued})" if dma_on else "s_waitcnt vmcnt(0)"]
        gaps[67] += ["s_barrier"]  # tile t+1 landed for every wave
    if read_next:
        gaps[67] += ["v_xor_b32 %[va], %[vax], %[va]", "v_xor_b32 %[vb], %[vbx], %[vb]"]
        reads_h0 = [frag_half(B_BASE, f, 0, "%[vb]") for f in range(8)] + [frag_half(A_BASE, f, 0, "%[va]") for f in range(8)]
        for n, r in enumerate(reads_h0):
            gaps[68 + 3 * n + (1 if n % 2 else 0)] += [r]
        gaps[127] += ["s_waitcnt lgkmcnt(0)"]
    lines = []
    for h in range(2):
        for i in range(8):
            for j in range(8):
                g = 64 * h + 8 * i + j
                lines.append(mfma_bf16(i, j, h))
                lines += gaps[g]
    return lines


def main_loop_kh():
    L = setup(2)
    L.append(f"s_mov_b32 s{CNT}, %[cnt]")
    for a in range(256):
        L.append(f"v_accvgpr_write_b32 a{a}, 0")
    L += ["s_waitcnt vmcnt(16)", "s_barrier"]
    L += [frag_half(B_BASE, f, 0, "%[vb]") for f in range(8)] + [frag_half(A_BASE, f, 0, "%[va]") for f in range(8)]
    L += ["s_waitcnt lgkmcnt(0)"]
    L += [f"s_cmp_eq_u32 s{CNT}, 0", "s_cbranch_scc1 2f", "1:"]
    L += body_kh(True, True, True)
    L += [f"s_sub_u32 s{CNT}, s{CNT}, 1", f"s_cmp_eq_u32 s{CNT}, 0", "s_cbranch_scc0 1b", "2:"]
    L += body_kh(False, True, True)
    L += body_kh(False, False, False)
    L += ["s_nop 7", "s_nop 7", "s_nop 7", f"s_mov_b32 m0, s{M0_KEEP}"]
    return L


def setup(k_tiles_skipped: int, amn: bool = False, bmn: bool = False, mn8: bool = False):
    """SRDs at K-tile `k_tiles_skipped` of this tile's A / B rows, soffsets, DMA destinations of buffer 0. fp8 MN-major
    operands (`mn8`): %[stride] / %[stridea] are the row strides in bytes, the soffsets MN8_ROW_OFF[j] rows, and B's DMA
    base comes in as %[m0b] (the two images have different chunk strides)."""
    L = [f"s_mov_b32 s{M0_KEEP}, m0",
         f"s_mov_b64 s[{SRD_A}:{SRD_A + 1}], %[pa]", f"s_mov_b32 s{SRD_A + 2}, -1", f"s_mov_b32 s{SRD_A + 3}, 0x20000",
         f"s_mov_b64 s[{SRD_B}:{SRD_B + 1}], %[pb]", f"s_mov_b32 s{SRD_B + 2}, -1", f"s_mov_b32 s{SRD_B + 3}, 0x20000"]
    if bmn and mn8:
        L += [f"s_mul_i32 s{SOFF + n - 1}, %[stride], {MN8_ROW_OFF[n - 1]}" for n in range(1, 8)]
    else:
        L.append(f"s_mov_b32 s{SOFF}, %[stride]")
        for n in range(1, 7):
            L.append(f"s_add_u32 s{SOFF + n}, s{SOFF + n - 1}, %[stride]")
    if amn and mn8:
        L += [f"s_mov_b32 s{ADV_A}, %[adva]"]
        L += [f"s_mul_i32 s{SOFF_A + n - 1}, %[stridea], {MN8_ROW_OFF[n - 1]}" for n in range(1, 8)]
    elif amn:
        L += [f"s_mov_b32 s{SOFF_A}, %[stridea]", f"s_mov_b32 s{ADV_A}, %[adva]"]
        for n in range(1, 7):
            L.append(f"s_add_u32 s{SOFF_A + n}, s{SOFF_A + n - 1}, %[stridea]")
    if bmn:
        L += [f"s_mov_b32 s{ADV_B}, %[advb]"]
    for _ in range(k_tiles_skipped):
        L += advance_srd("A", amn) + advance_srd("B", bmn)
    L += [f"s_mov_b32 s{M0_A}, %[m0a]", f"s_mov_b32 s{M0_B}, %[m0b]" if mn8 else f"s_add_u32 s{M0_B}, %[m0a], 33792",
          f"s_add_u32 s{M0_X}, %[m0a], 67584", f"s_xor_b32 s{M0_X}, s{M0_X}, %[m0a]",
          f"s_add_u32 s{M0_XB}, s{M0_B}, 67584", f"s_xor_b32 s{M0_XB}, s{M0_XB}, s{M0_B}"]
    return L


def issue(amn: bool = False, bmn: bool = False, mn8: bool = False):
    """DMA of K-tiles 0 and 1 of a tile into LDS buffers 0 and 1. Issued for the NEXT tile of a persistent
    workgroup before the current tile's epilogue (every wave passed the last body's final barrier after its last
    ds_read, so both buffers are free), which hides the first loads' latency under the epilogue."""
    L = setup(0, amn, bmn, mn8)
    for tile in range(2):
        L.append(f"s_mov_b32 m0, s{M0_B}")
        L.append("s_nop 0")
        for n in range(8):
            L += dma("B", n, bmn, mn8)
        L.append(f"s_mov_b32 m0, s{M0_A}")
        L.append("s_nop 0")
        for n in range(8):
            L += dma("A", n, amn, mn8)
        if tile == 0:
            L += advance_srd("A", amn) + advance_srd("B", bmn)
            L += [f"s_xor_b32 s{M0_A}, s{M0_A}, s{M0_X}", f"s_xor_b32 s{M0_B}, s{M0_B}, s{M0_XB}"]
    L.append(f"s_mov_b32 m0, s{M0_KEEP}")
    return L


def main_loop(bf16: bool = False, amn: bool = False, bmn: bool = False, probe: str = "", mn8: bool = False):
    """Everything after `issue()`: zero the accumulators, K-tile 0's fragments, the loop and the 2-tile tail.
    vmcnt(16) at the start: the 32 DMAs of `issue()` plus whatever epilogue stores the previous tile issued after
    them (vmcnt counts in order) -> at most the 16 newest may still be in flight, so K-tile 0 has landed."""
    L = setup(2, amn, bmn, mn8)
    L.append(f"s_mov_b32 s{CNT}, %[cnt]")
    for a in range(256):
        L.append(f"v_accvgpr_write_b32 a{a}, 0")
    L += ["s_waitcnt vmcnt(16)", "s_barrier"]
    for f in range(4):
        L += b_frag(f, bmn, mn8)
    for f in range(4):
        L += a_frag(f, amn, mn8)
    L += ["s_waitcnt lgkmcnt(0)"]
    L += [f"s_cmp_eq_u32 s{CNT}, 0", "s_cbranch_scc1 2f", "1:"]
    # probe loops (timing diagnostics only, wrong results): "nodma" issues no LDS-DMA inside the loop, "noread" no
    # fragment reads, "mfma" neither
    L += body(dma_on=probe not in ("nodma", "mfma"), wait_next=True, read_next=True, bf16=bf16, amn=amn, bmn=bmn,
              reads_on=probe not in ("noread", "mfma"), mn8=mn8)
    L += [f"s_sub_u32 s{CNT}, s{CNT}, 1", f"s_cmp_eq_u32 s{CNT}, 0", "s_cbranch_scc0 1b", "2:"]
    L += body(dma_on=False, wait_next=True, read_next=True, bf16=bf16, amn=amn, bmn=bmn, mn8=mn8)
    L += body(dma_on=False, wait_next=False, read_next=False, bf16=bf16, amn=amn, bmn=bmn, mn8=mn8)
    L += ["s_nop 7", "s_nop 7", "s_nop 7", f"s_mov_b32 m0, s{M0_KEEP}"]
    return L


# ---------------------------------------------------------------------------------------------------- 8-wave loop
# Two waves per SIMD (512-thread workgroup): wave (wm, wn), wm = 0..3, owns a 64 x 128 block = 4 x 8 accumulator
# blocks (a[0:127]); fragments A0-3 in v[32:63], B0-7 in v[64:127] (256 registers per lane: AGPRs + VGPRs). The K-loop
# has the 4-wave loop's shape (same LDS image, 3 barriers per K-tile, quadrant order A0-1 x B0-3 | A0-1 x B4-7 |
# A2-3 x B0-3 | A2-3 x B4-7 with the next fragments read into the dead registers), but each wave issues half the
# MFMAs and half the LDS-DMA (4 A + 4 B per K-tile): the 4-wave probes (tools/bench_gemm_probe.py) put ~15 % of the
# loop in DMA issue, which a second wave on the SIMD can cover with its MFMAs.
# A fragment i of lane (r, g) = slab row 8 (r >> 1) + (r & 1) + 2 i: lanes r, r ^ 1 share a chunk 128 B apart and the
# 16-lane ds_read_b128 groups land on 16 distinct 16-B bank slots.
A8_BASE, B8_BASE = 32, 64
CHUNK8_STEP = 8 * 1056  # m0 advance per DMA instruction (8 waves x one chunk)


def w8_a(i):
    return f"v[{A8_BASE + 8 * i}:{A8_BASE + 8 * i + 7}]"


def w8_b(j):
    return f"v[{B8_BASE + 8 * j}:{B8_BASE + 8 * j + 7}]"


def w8_mfma(i, j):
    return f"v_mfma_f32_16x16x128_f8f6f4 {acc(i, j)}, {w8_a(i)}, {w8_b(j)}, {acc(i, j)} cbsz:%c[fa] blgp:%c[fb]"


def w8_mfma_bf16(i, j, half):
    a0, b0 = A8_BASE + 8 * i + 4 * half, B8_BASE + 8 * j + 4 * half
    return f"v_mfma_f32_16x16x32_bf16 {acc(i, j)}, v[{a0}:{a0 + 3}], v[{b0}:{b0 + 3}], {acc(i, j)}"


def w8_afrag(i):
    d = A8_BASE + 8 * i
    return [f"ds_read_b128 v[{d}:{d + 3}], %[va] offset:{256 * i}", f"ds_read_b128 v[{d + 4}:{d + 7}], %[va] offset:{256 * i + 64}"]


def w8_bfrag(j):
    d = B8_BASE + 8 * j
    return [f"ds_read_b128 v[{d}:{d + 3}], %[vb] offset:{128 * j}", f"ds_read_b128 v[{d + 4}:{d + 7}], %[vb] offset:{128 * j + 64}"]


def w8_dma(op, n):
    srd = SRD_A if op == "A" else SRD_B
    so = "0" if n == 0 else f"s{SOFF + n - 1}"
    out = [f"buffer_load_dwordx4 %[voff], s[{srd}:{srd + 3}], {so} offen lds"]
    if n < 3:
        out.append(f"s_add_u32 m0, m0, {CHUNK8_STEP}")
    return out


def w8_body(dma_on: bool, wait_next: bool, read_next: bool, bf16: bool):
    slots = {k: [] for k in range(32)}
    order = ([(i, j) for i in range(2) for j in range(4)] + [(i, j) for i in range(2) for j in range(4, 8)]
             + [(i, j) for i in range(2, 4) for j in range(4)] + [(i, j) for i in range(2, 4) for j in range(4, 8)])
    for f in range(4):  # Q1: B4-7 of t
        slots[f] += w8_bfrag(4 + f)
    if dma_on:
        slots[4] += [f"s_mov_b32 m0, s{M0_B}"]
    slots[4] += ["s_waitcnt lgkmcnt(0)"]
    slots[5] += ["s_barrier"]  # every wave holds all of B(t): B(t+2) may overwrite the buffer
    if dma_on:
        for n in range(4):
            slots[6 + n] += w8_dma("B", n)
    slots[10] += w8_afrag(2)  # Q2: A2-3 of t
    slots[11] += w8_afrag(3)
    if dma_on:
        slots[12] += advance_srd("B")
    slots[13] += ["s_waitcnt lgkmcnt(0)"]
    slots[14] += ["s_barrier"]  # every wave holds all of A(t)
    if dma_on:
        slots[15] += [f"s_mov_b32 m0, s{M0_A}"]
        for n in range(4):
            slots[16 + n] += w8_dma("A", n)
        slots[20] += advance_srd("A")
    if wait_next:
        slots[22] += ["s_waitcnt vmcnt(8)" if dma_on else "s_waitcnt vmcnt(0)"]
        slots[23] += ["s_barrier"]  # K-tile t+1 landed for every wave
    if read_next:  # Q4: B0-3 and A0-1 of t+1 from the other buffer
        slots[24] += ["v_xor_b32 %[va], %[vax], %[va]", "v_xor_b32 %[vb], %[vbx], %[vb]"]
        for f in range(4):
            slots[24 + f] += w8_bfrag(f)
        slots[28] += w8_afrag(0)
        slots[29] += w8_afrag(1)
    if dma_on:
        slots[30] += [f"s_xor_b32 s{M0_A}, s{M0_A}, s{M0_X}", f"s_xor_b32 s{M0_B}, s{M0_B}, s{M0_XB}"]
    if read_next:
        slots[31] += ["s_waitcnt lgkmcnt(0)"]
    lines = []
    if not bf16:
        for k, (i, j) in enumerate(order):
            lines.append(w8_mfma(i, j))
            lines += slots[k]
        return lines
    for c in range(0, 32, 4):
        for k in range(c, c + 4):
            lines.append(w8_mfma_bf16(*order[k], 0))
            lines += slots[k]
        for k in range(c, c + 4):
            lines.append(w8_mfma_bf16(*order[k], 1))
    return lines


def w8_setup(k_tiles_skipped: int):
    L = [f"s_mov_b32 s{M0_KEEP}, m0",
         f"s_mov_b64 s[{SRD_A}:{SRD_A + 1}], %[pa]", f"s_mov_b32 s{SRD_A + 2}, -1", f"s_mov_b32 s{SRD_A + 3}, 0x20000",
         f"s_mov_b64 s[{SRD_B}:{SRD_B + 1}], %[pb]", f"s_mov_b32 s{SRD_B + 2}, -1", f"s_mov_b32 s{SRD_B + 3}, 0x20000",
         f"s_mov_b32 s{SOFF}, %[stride]", f"s_add_u32 s{SOFF + 1}, s{SOFF}, %[stride]", f"s_add_u32 s{SOFF + 2}, s{SOFF + 1}, %[stride]"]
    for _ in range(k_tiles_skipped):
        L += advance_srd("A") + advance_srd("B")
    L += [f"s_mov_b32 s{M0_A}, %[m0a]", f"s_add_u32 s{M0_B}, %[m0a], 33792",
          f"s_add_u32 s{M0_X}, %[m0a], 67584", f"s_xor_b32 s{M0_X}, s{M0_X}, %[m0a]",
          f"s_add_u32 s{M0_XB}, s{M0_B}, 67584", f"s_xor_b32 s{M0_XB}, s{M0_XB}, s{M0_B}"]
    return L


def w8_issue():
    L = w8_setup(0)
    for tile in range(2):
        L += [f"s_mov_b32 m0, s{M0_B}", "s_nop 0"]
        for n in range(4):
            L += w8_dma("B", n)
        L += [f"s_mov_b32 m0, s{M0_A}", "s_nop 0"]
        for n in range(4):
            L += w8_dma("A", n)
        if tile == 0:
            L += advance_srd("A") + advance_srd("B")
            L += [f"s_xor_b32 s{M0_A}, s{M0_A}, s{M0_X}", f"s_xor_b32 s{M0_B}, s{M0_B}, s{M0_XB}"]
    L.append(f"s_mov_b32 m0, s{M0_KEEP}")
    return L


def w8_main_loop(bf16: bool):
    L = w8_setup(2)
    L.append(f"s_mov_b32 s{CNT}, %[cnt]")
    for a in range(128):
        L.append(f"v_accvgpr_write_b32 a{a}, 0")
    L += ["s_waitcnt vmcnt(8)", "s_barrier"]
    for f in range(4):
        L += w8_bfrag(f)
    L += w8_afrag(0) + w8_afrag(1)
    L += ["s_waitcnt lgkmcnt(0)"]
    L += [f"s_cmp_eq_u32 s{CNT}, 0", "s_cbranch_scc1 2f", "1:"]
    L += w8_body(True, True, True, bf16)
    L += [f"s_sub_u32 s{CNT}, s{CNT}, 1", f"s_cmp_eq_u32 s{CNT}, 0", "s_cbranch_scc0 1b", "2:"]
    L += w8_body(False, True, True, bf16)
    L += w8_body(False, False, False, bf16)
    L += ["s_nop 7", "s_nop 7", "s_nop 7", f"s_mov_b32 m0, s{M0_KEEP}"]
    return L


def generate() -> str:
    I, L, LB = issue(), main_loop(), main_loop(bf16=True)
    SPREAD[0] = True  # the MN-major bf16 loops (weight gradients, default) in the spread issue order
    IT, LT = issue(amn=True), main_loop(bf16=True, amn=True)
    IBT, LBT = issue(amn=True, bmn=True), main_loop(bf16=True, amn=True, bmn=True)
    LS8 = main_loop(bf16=False, probe="")  # fp8 K-major loop, spread order (FP8ASM_SPREAD_MAIN_LOOP)
    SPREAD[0] = False
    probes = [(f"BF16ASM_PROBE_{k.upper()}_LOOP", main_loop(bf16=True, probe=k)) for k in ("nodma", "noread", "mfma")]
    for k in ("regload", "regstage"):
        PROBE_LOADS[0] = k
        probes.append((f"BF16ASM_PROBE_{k.upper()}_LOOP", main_loop(bf16=True)))
        PROBE_LOADS[0] = None
    SPREAD[0] = True
    probes.append(("BF16ASM_SPREAD_MAIN_LOOP", main_loop(bf16=True)))
    SPREAD[0] = False
    probes.append(("BF16ASM_KH_MAIN_LOOP", main_loop_kh()))
    assert sum(1 for x in probes[-1][1] if x.startswith("v_mfma")) == 3 * 128
    assert sum(1 for x in probes[-1][1] if x.startswith("v_mfma")) == 3 * 128
    f8mn = [("FP8AMN_ISSUE", issue(amn=True, mn8=True)), ("FP8AMN_MAIN_LOOP", main_loop(amn=True, mn8=True)),
            ("FP8ABMN_ISSUE", issue(amn=True, bmn=True, mn8=True)),
            ("FP8ABMN_MAIN_LOOP", main_loop(amn=True, bmn=True, mn8=True))]
    assert sum(1 for x in f8mn[3][1] if x.startswith("ds_read_b64_tr_b8")) == 2 * (16 + 32 + 32 + 16)
    w8 = [("W8_ISSUE", w8_issue()), ("W8_BF16_MAIN_LOOP", w8_main_loop(True)), ("W8_FP8_MAIN_LOOP", w8_main_loop(False))]
    assert sum(1 for x in w8[1][1] if x.startswith("v_mfma")) == 3 * 64
    assert sum(1 for x in w8[2][1] if x.startswith("v_mfma")) == 3 * 32
    assert sum(1 for x in LBT if x.startswith("ds_read_b64_tr_b16")) == 2 * (16 + 32 + 32 + 16)
    n_mfma = sum(1 for x in L if x.startswith("v_mfma"))
    assert n_mfma == 3 * 64, n_mfma
    assert sum(1 for x in LB if x.startswith("v_mfma")) == 3 * 128
    assert sum(1 for x in LT if x.startswith("v_mfma")) == 3 * 128
    assert sum(1 for x in LT if x.startswith("ds_read_b64_tr_b16")) == 16 + 32 + 32 + 16
    out = ["// GENERATED by tools/gen_fp8_asm.py -- do not edit by hand; edit the generator and rerun it.",
           "// K-loop of fp8_gemm_asm_kernel (csrc/kernels/fp8_gemm_asm.hip): see the generator's docstring.",
           f"// FP8ASM_ISSUE {len(I)} lines; FP8ASM_MAIN_LOOP {len(L)} lines, {n_mfma} MFMAs (loop body 64);",
           f"// BF16ASM_MAIN_LOOP {len(LB)} lines (loop body 128 MFMAs); BF16AMN_* (MN-major A): {len(IT)} / {len(LT)} lines.",
           "#pragma once"]
    for name, lines in (("FP8ASM_ISSUE", I), ("FP8ASM_MAIN_LOOP", L), ("FP8ASM_SPREAD_MAIN_LOOP", LS8), ("BF16ASM_MAIN_LOOP", LB),
                        ("BF16AMN_ISSUE", IT), ("BF16AMN_MAIN_LOOP", LT),
                        ("BF16ABMN_ISSUE", IBT), ("BF16ABMN_MAIN_LOOP", LBT)) + tuple(probes) + tuple(f8mn) + tuple(w8):
        out.append(f"#define {name} \\")
        for x in lines:
            out.append(f'  "{x}\\n" \\')
        out.append('  ""')
        out.append("")
    out.append(f"#define FP8ASM_SGPR_CLOBBERS " + ", ".join(f'"s{s}"' for s in range(SRD_A, M0_KEEP + 1)))
    out.append(f"#define BF16AMN_SGPR_CLOBBERS " + ", ".join(f'"s{s}"' for s in range(SRD_A, ADV_A + 1)))
    out.append(f"#define BF16ABMN_SGPR_CLOBBERS " + ", ".join(f'"s{s}"' for s in range(SRD_A, ADV_B + 1)))
    out.append(f"#define W8_VCLOBBERS " + ", ".join(f'"v{v}"' for v in range(A8_BASE, 128)))
    out.append(f"#define W8_ACLOBBERS " + ", ".join(f'"a{a}"' for a in range(128)))
    out.append("")
    return "\n".join(out)


def main(argv):
    here = os.path.dirname(os.path.abspath(__file__))
    path = os.path.join(here, "..", "accelerate_hpc_test_amd", "csrc", "kernels", "fp8_asm_loop.inc")
    text = generate()
    if len(argv) > 1 and argv[1] == "--check":
        with open(path) as f:
            return 0 if f.read() == text else 1
    with open(path, "w") as f:
        f.write(text)
    print(f"wrote {os.path.normpath(path)}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
