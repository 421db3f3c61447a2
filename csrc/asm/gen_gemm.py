#!/usr/bin/env python3
"""Generator of the hand-scheduled CDNA4 (gfx950) GEMM kernels in assembly.

    C[M, N] = A[M, K] . B[N, K]^T       (both operands K-contiguous, bf16 in, fp32 accumulate)

Why assembly: rounds 2-4 showed that a one-wave-per-SIMD GEMM (the register layout hipBLASLt's fastest
gfx950 kernels use: 4 waves, a 128 x 128 fp32 quadrant per wave in AGPRs) does not reach the library's
main loop in HIP source -- hipcc sinks fragment reads to their first use, waits ``lgkmcnt(0)`` before each
MFMA row and drains the LDS-DMA queue at barriers (``profiles/r3_gemm_w4.txt``).  Here every instruction is
placed by this script, so the schedule is exactly the one designed below.

Design (one 256-thread workgroup per CU, persistent over output tiles):

* Tile 256 x 256, K-step 64.  Wave ``q`` (0..3) owns the quadrant (wm, wn) = (q >> 1, q & 1): 8 x 8
  ``v_mfma_f32_16x16x32_bf16`` accumulators = 256 AGPRs; 128 MFMAs per K-step per wave.
* LDS: two 64 KB stages {A image 32 KB | B image 32 KB}.  An operand image is 32 "pieces" of 1 KB, one per
  (wave half w, fragment f, k-half h): piece lane ``t = p + 16 u`` holds row ``p`` of fragment f, k-chunk
  ``4 h + u`` (16 bytes).  A fragment read is then ONE linear 1 KB ``ds_read_b128`` at ``piece + 16 lane``
  -- bank-conflict free with no swizzle -- and the LDS-DMA (``buffer_load_dwordx4 ... lds``, which writes
  lane-linearly) fills a piece with one instruction whose per-lane global addresses do the layout work.
* B fragment f covers output columns ``8 c + f`` (c = lane & 15): after the MFMA each lane holds, for one
  output row, 8 CONSECUTIVE columns across its 8 column fragments, so the epilogue writes 16 bytes per lane
  and 8 whole 128-byte lines per store instruction with no cross-lane exchange.
* Pipeline (per K-step t, stage X = t & 1): the k-half-1 fragments of step t are read into the second
  register set under the first 32 MFMAs (k-half 0 set); barrier B2 (everyone's reads of stage X retired)
  then the LDS-DMA of step t + 2 is issued INTO stage X under the next MFMAs (two steps ahead in two
  stages: a stage is refilled as soon as its last reads retire); ``vmcnt(16)`` + barrier B3 (step t + 1's
  DMA landed everywhere) and the k-half-0 fragments of step t + 1 are read from stage Y under the last 32
  MFMAs.  Two barriers per 128 MFMAs; no MFMA waits on a fragment read.
* Output mapping per lane l (c = l & 15, g = l >> 4), fragment (i, j), register r:
  ``C[row0 + 128 wm + 16 i + 4 g + r][col0 + 128 wn + 8 c + j]``.

Epilogues (``EPI``): ``plain`` (bf16 C), ``bias`` (bf16 C + fp32 bias[n]).

Usage:  gen_gemm.py OUT.s      (assemble with clang -target amdgcn-amd-amdhsa -mcpu=gfx950)
"""
import sys

# ----------------------------------------------------------------------------------------------------
# register map
# ----------------------------------------------------------------------------------------------------
# SGPRs
S_KARG = 0          # s[0:1] kernarg pointer
S_WG = 2            # workgroup id
S_A, S_B, S_C, S_AUX0 = 4, 6, 8, 10   # 64-bit pointers
S_M, S_N, S_K, S_LDA, S_LDB, S_LDC, S_TN, S_NT, S_GRID = 12, 13, 14, 15, 16, 17, 18, 19, 20
S_SRDA, S_SRDB, S_SRDC = 24, 28, 32   # buffer resources (4 SGPRs each)
S_OFFA = 36         # 8 soffsets of the A pieces (s36..s43)
S_OFFB = 44         # 8 soffsets of the B pieces (s44..s51)
S_TILE = 52         # current tile id
S_KT = 53           # K-steps per tile
S_LOOP = 54         # loop counter
S_MBASE = 55        # LDS-DMA base of this wave's pieces in the stage being refilled (stage X)
S_WAVE = 56         # wave id
S_ROW0, S_COL0 = 57, 58
S_NRA, S_NRB = 59, 60   # remaining num_records of the A / B resources
S_LDC2 = 61         # ldc * 2
S_T0, S_T1, S_T2, S_T3 = 62, 63, 64, 65
S_SOFFC = 66
S_AUXP = 68         # s[68:69] aux pointer of the current tile (bias + col0)
S_SRDX = 72         # s[72:75] a spare resource (epilogue operands)
S_LAST = 80

# VGPRs
V_TID = 0
V_GA, V_GB = 1, 2            # per-lane LDS-DMA global offsets (A, B)
V_RA, V_RB = 3, 4            # per-lane ds_read bases (stage X)
V_CO = 5                     # per-lane epilogue C offset
V_T = 6                      # temps v6, v7
SET0_A, SET0_B, SET1_A, SET1_B = 8, 40, 72, 104   # 4 fragment register blocks of 32 VGPRs
V_EPI = 136                  # epilogue scratch v136..v255
V_BIAS = 248                 # 8 bias values per lane (v248..v255)

STAGE = 65536
B_IMG = 32768
PIECE = 1024


class Emitter:
    def __init__(self, prefix=""):
        self.lines = []
        self.nlabel = 0
        self.prefix = prefix

    def L(self, stem):
        """a kernel-local label name"""
        return f".L{self.prefix}_{stem}"

    def __call__(self, s):
        self.lines.append("\t" + s)

    def label(self, name):
        self.lines.append(f"{name}:")

    def fresh(self, stem):
        self.nlabel += 1
        return f".L{self.prefix}_{stem}_{self.nlabel}"

    def text(self):
        return "\n".join(self.lines) + "\n"


def vr(base, n=4):
    return f"v[{base}:{base + n - 1}]"


def sr(base, n):
    return f"s[{base}:{base + n - 1}]" if n > 1 else f"s{base}"


def acc(i, j):
    b = (i * 8 + j) * 4
    return f"a[{b}:{b + 3}]"


# ----------------------------------------------------------------------------------------------------
# main-loop building blocks
# ----------------------------------------------------------------------------------------------------
def mfma_list(set_a, set_b, zero_c):
    """the 64 MFMAs of one k-half (i-major), as instruction strings"""
    out = []
    for i in range(8):
        for j in range(8):
            c = "0" if zero_c else acc(i, j)
            out.append(f"v_mfma_f32_16x16x32_bf16 {acc(i, j)}, {vr(set_a + 4 * i)}, {vr(set_b + 4 * j)}, {c}")
    return out


def frag_reads(set_a, set_b, base_a_v, base_b_v, h):
    """16 ds_read_b128: 8 A fragments and 8 B fragments of k-half h (pieces 2f + h of the wave half)"""
    out = []
    for f in range(8):
        out.append(f"ds_read_b128 {vr(set_a + 4 * f)}, v{base_a_v} offset:{(2 * f + h) * PIECE}")
        out.append(f"ds_read_b128 {vr(set_b + 4 * f)}, v{base_b_v} offset:{(2 * f + h) * PIECE}")
    return out


def glds_list():
    """16 LDS-DMA pieces of one K-step: this wave's A pieces 8q+s then its B pieces 8q+s (s = 0..7).
    M0 = S_MBASE (+ B_IMG) + s * 1KB; each load is preceded by its M0 write (one SALU between is enough)."""
    out = []
    for s in range(8):
        out.append([f"s_add_u32 m0, s{S_MBASE}, {s * PIECE}", "s_nop 0",
                    f"buffer_load_dwordx4 v{V_GA}, {sr(S_SRDA, 4)}, s{S_OFFA + s} offen lds"])
    for s in range(8):
        out.append([f"s_add_u32 m0, s{S_MBASE}, {B_IMG + s * PIECE}", "s_nop 0",
                    f"buffer_load_dwordx4 v{V_GB}, {sr(S_SRDB, 4)}, s{S_OFFB + s} offen lds"])
    return out


def advance_k():
    """move both operand resources one K-step (128 bytes) forward"""
    return [
        f"s_add_u32 s{S_SRDA}, s{S_SRDA}, 128", f"s_addc_u32 s{S_SRDA + 1}, s{S_SRDA + 1}, 0",
        f"s_sub_u32 s{S_NRA}, s{S_NRA}, 128", f"s_mov_b32 s{S_SRDA + 2}, s{S_NRA}",
        f"s_add_u32 s{S_SRDB}, s{S_SRDB}, 128", f"s_addc_u32 s{S_SRDB + 1}, s{S_SRDB + 1}, 0",
        f"s_sub_u32 s{S_NRB}, s{S_NRB}, 128", f"s_mov_b32 s{S_SRDB + 2}, s{S_NRB}",
    ]


def iteration(e, kind):
    """one K-step.  kind: 'first' (zero-init accumulators, DMA t+2), 'loop' (DMA t+2),
    'penult' (no DMA, wait all), 'last' (no DMA, no next reads).
    Entry: SET0 holds this step's k-half-0 fragments (waited); V_RA/V_RB point at stage X."""
    m0 = mfma_list(SET0_A, SET0_B, kind == "first")
    m1 = mfma_list(SET1_A, SET1_B, False)
    slots = [[] for _ in range(128)]  # instructions issued after MFMA n

    # k-half-1 fragments of this step (stage X) under MFMAs 0..31
    for n, ins in enumerate(frag_reads(SET1_A, SET1_B, V_RA, V_RB, 1)):
        slots[2 * n].append(ins)
    dma = kind in ("first", "loop")
    if dma:
        # B2 after the k-half-1 reads retired: stage X is free; refill it with step t + 2
        slots[36].append("s_waitcnt lgkmcnt(0)")
        slots[36].append("s_barrier")
        for n, grp in enumerate(glds_list()):
            slots[38 + 3 * n].extend(grp)     # 38 .. 83
        slots[86].extend(advance_k())
    else:
        slots[40].append("s_waitcnt lgkmcnt(0)")
    if kind != "last":
        # B3: step t + 1's DMA landed for every wave, then read its k-half-0 fragments from stage Y
        slots[90].append("s_waitcnt vmcnt(16)" if dma else "s_waitcnt vmcnt(0)")
        slots[90].append("s_barrier")
        slots[90].append(f"v_xor_b32 v{V_RA}, {STAGE}, v{V_RA}")
        slots[90].append(f"v_xor_b32 v{V_RB}, {STAGE}, v{V_RB}")
        slots[90].append(f"s_xor_b32 s{S_MBASE}, {STAGE}, s{S_MBASE}")
        for n, ins in enumerate(frag_reads(SET0_A, SET0_B, V_RA, V_RB, 0)):
            slots[92 + 2 * n].append(ins)     # 92 .. 122
        slots[127].append("s_waitcnt lgkmcnt(0)")
    mf = m0 + m1
    for n in range(128):
        e(mf[n])
        for ins in slots[n]:
            e(ins)


# ----------------------------------------------------------------------------------------------------
# kernel
# ----------------------------------------------------------------------------------------------------
def kernel(name, epi):
    e = Emitter(name)
    # ---- arguments ----
    e(f"s_load_dwordx8 {sr(S_A, 8)}, s[0:1], 0x0")          # A B C AUX0
    e(f"s_load_dwordx8 {sr(S_M, 8)}, s[0:1], 0x30")         # M N K lda ldb ldc tiles_n num_tiles
    e(f"s_load_dword s{S_GRID}, s[0:1], 0x50")
    e(f"v_lshrrev_b32 v{V_T}, 6, v{V_TID}")
    e(f"v_readfirstlane_b32 s{S_WAVE}, v{V_T}")
    e("s_waitcnt lgkmcnt(0)")
    # K-steps, ldc*2
    e(f"s_lshr_b32 s{S_KT}, s{S_K}, 6")
    e(f"s_lshl_b32 s{S_LDC2}, s{S_LDC}, 1")
    # the K-step schedule needs at least 4 steps (first, loop >= 1, penult, last): never loop on less
    e(f"s_cmp_lt_u32 s{S_KT}, 4")
    e("s_cbranch_scc1 " + e.L("end"))
    # ---- per-lane LDS-DMA offsets ----
    # A: row = 128 (q >> 1) + 64 (q & 1) + (t & 15), chunk = t >> 4
    # B: row = 128 (q >> 1) + 4 (q & 1) + 8 (t & 15), chunk = t >> 4
    e(f"s_lshr_b32 s{S_T0}, s{S_WAVE}, 1")
    e(f"s_lshl_b32 s{S_T0}, s{S_T0}, 7")                    # 128 (q >> 1)
    e(f"s_and_b32 s{S_T1}, s{S_WAVE}, 1")
    e(f"s_lshl_b32 s{S_T2}, s{S_T1}, 6")
    e(f"s_add_u32 s{S_T2}, s{S_T2}, s{S_T0}")               # A row base
    e(f"s_lshl_b32 s{S_T3}, s{S_T1}, 2")
    e(f"s_add_u32 s{S_T3}, s{S_T3}, s{S_T0}")               # B row base
    e(f"v_and_b32 v{V_T}, 15, v{V_TID}")                    # t & 15 (lane, since waves are 64 wide)
    e(f"v_add_u32 v{V_T + 1}, s{S_T2}, v{V_T}")              # A row
    e(f"s_lshl_b32 s{S_T0}, s{S_LDA}, 1")
    e(f"v_mul_lo_u32 v{V_GA}, v{V_T + 1}, s{S_T0}")
    e(f"v_lshlrev_b32 v{V_T + 1}, 3, v{V_T}")
    e(f"v_add_u32 v{V_T + 1}, s{S_T3}, v{V_T + 1}")          # B row
    e(f"s_lshl_b32 s{S_T1}, s{S_LDB}, 1")
    e(f"v_mul_lo_u32 v{V_GB}, v{V_T + 1}, s{S_T1}")
    e(f"v_lshrrev_b32 v{V_T}, 4, v{V_TID}")
    e(f"v_and_b32 v{V_T}, 3, v{V_T}")                        # (t >> 4) & 3 = chunk within the k-half
    e(f"v_lshlrev_b32 v{V_T}, 4, v{V_T}")
    e(f"v_add_u32 v{V_GA}, v{V_GA}, v{V_T}")
    e(f"v_add_u32 v{V_GB}, v{V_GB}, v{V_T}")
    # piece soffsets: A (s>>1)*16 rows + (s&1)*64 B; B (s>>1) rows + (s&1)*64 B
    for s in range(8):
        e(f"s_mul_i32 s{S_OFFA + s}, s{S_T0}, {16 * (s >> 1)}")
        if s & 1:
            e(f"s_add_u32 s{S_OFFA + s}, s{S_OFFA + s}, 64")
        e(f"s_mul_i32 s{S_OFFB + s}, s{S_T1}, {s >> 1}")
        if s & 1:
            e(f"s_add_u32 s{S_OFFB + s}, s{S_OFFB + s}, 64")
    # ---- per-lane fragment read bases (stage 0): A piece wm*16, B piece wn*16, + 16 lane ----
    e(f"v_and_b32 v{V_T}, 63, v{V_TID}")
    e(f"v_lshlrev_b32 v{V_T}, 4, v{V_T}")
    e(f"s_lshr_b32 s{S_T0}, s{S_WAVE}, 1")
    e(f"s_lshl_b32 s{S_T0}, s{S_T0}, 14")                   # wm * 16 KB
    e(f"v_add_u32 v{V_RA}, s{S_T0}, v{V_T}")
    e(f"s_and_b32 s{S_T1}, s{S_WAVE}, 1")
    e(f"s_lshl_b32 s{S_T1}, s{S_T1}, 14")
    e(f"s_add_u32 s{S_T1}, s{S_T1}, {B_IMG}")
    e(f"v_add_u32 v{V_RB}, s{S_T1}, v{V_T}")
    # ---- per-lane epilogue offset: row 128 wm + 4 g, col 128 wn + 8 c (bytes, relative to the tile) ----
    e(f"v_lshrrev_b32 v{V_T}, 4, v{V_TID}")
    e(f"v_and_b32 v{V_T}, 3, v{V_T}")
    e(f"v_lshlrev_b32 v{V_T}, 2, v{V_T}")                    # 4 g
    e(f"s_lshr_b32 s{S_T0}, s{S_WAVE}, 1")
    e(f"s_lshl_b32 s{S_T0}, s{S_T0}, 7")
    e(f"v_add_u32 v{V_T}, s{S_T0}, v{V_T}")                  # row
    e(f"v_mul_lo_u32 v{V_CO}, v{V_T}, s{S_LDC2}")
    e(f"v_and_b32 v{V_T}, 15, v{V_TID}")
    e(f"v_lshlrev_b32 v{V_T}, 4, v{V_T}")                    # 8 c columns * 2 bytes
    e(f"s_and_b32 s{S_T1}, s{S_WAVE}, 1")
    e(f"s_lshl_b32 s{S_T1}, s{S_T1}, 8")                    # 128 wn * 2 bytes
    e(f"v_add_u32 v{V_T}, s{S_T1}, v{V_T}")
    e(f"v_add_u32 v{V_CO}, v{V_CO}, v{V_T}")
    if epi == "bias":
        # byte offset of this lane's 8 bias values relative to col0: (128 wn + 8 c) * 4
        e(f"v_and_b32 v{V_T + 1}, 15, v{V_TID}")
        e(f"v_lshlrev_b32 v{V_T + 1}, 5, v{V_T + 1}")
        e(f"s_and_b32 s{S_T1}, s{S_WAVE}, 1")
        e(f"s_lshl_b32 s{S_T1}, s{S_T1}, 9")
        e(f"v_add_u32 v{V_T + 1}, s{S_T1}, v{V_T + 1}")
    # ---- tile loop: tile = round * grid + (wg % 8) * (grid / 8) + wg / 8 ----
    e(f"s_and_b32 s{S_T0}, s{S_WG}, 7")
    e(f"s_lshr_b32 s{S_T1}, s{S_GRID}, 3")
    e(f"s_mul_i32 s{S_T0}, s{S_T0}, s{S_T1}")
    e(f"s_lshr_b32 s{S_T1}, s{S_WG}, 3")
    e(f"s_add_u32 s{S_TILE}, s{S_T0}, s{S_T1}")
    e.label(e.L("tile"))
    e(f"s_cmp_lt_u32 s{S_TILE}, s{S_NT}")
    e("s_cbranch_scc0 " + e.L("end"))
    # tile coordinates: tm = tile / tiles_n, tn = tile % tiles_n (tiles_n is a power of two or not: use the
    # float-free unsigned division by repeated structure: tiles_n <= 64, so a 6-step restoring division)
    udiv(e, S_T0, S_TILE, S_TN, S_T1)           # S_T0 = tile / tiles_n ; S_T1 = remainder
    e(f"s_lshl_b32 s{S_ROW0}, s{S_T0}, 8")
    e(f"s_lshl_b32 s{S_COL0}, s{S_T1}, 8")
    # A resource: base = A + row0 * lda * 2, num_records = 256 * lda * 2
    set_srd(e, S_SRDA, S_A, S_ROW0, S_LDA, S_NRA)
    set_srd(e, S_SRDB, S_B, S_COL0, S_LDB, S_NRB)
    # C resource: base = C + (row0 * ldc + col0) * 2, num_records = 256 * ldc * 2
    e(f"s_mul_i32 s{S_T0}, s{S_ROW0}, s{S_LDC}")
    e(f"s_mul_hi_u32 s{S_T1}, s{S_ROW0}, s{S_LDC}")
    e(f"s_add_u32 s{S_T0}, s{S_T0}, s{S_COL0}")
    e(f"s_addc_u32 s{S_T1}, s{S_T1}, 0")
    e(f"s_lshl_b64 s[{S_T0}:{S_T1}], s[{S_T0}:{S_T1}], 1")
    e(f"s_add_u32 s{S_SRDC}, s{S_C}, s{S_T0}")
    e(f"s_addc_u32 s{S_SRDC + 1}, s{S_C + 1}, s{S_T1}")
    e(f"s_lshl_b32 s{S_SRDC + 2}, s{S_LDC2}, 8")
    e(f"s_mov_b32 s{S_SRDC + 3}, 0x20000")
    # stage-0 DMA base of this wave's pieces: q * 8 KB
    e(f"s_lshl_b32 s{S_MBASE}, s{S_WAVE}, 13")
    # prologue: K-steps 0 and 1 into stages 0 and 1
    for grp in glds_list():
        for ins in grp:
            e(ins)
    for ins in advance_k():
        e(ins)
    e(f"s_xor_b32 s{S_MBASE}, {STAGE}, s{S_MBASE}")
    for grp in glds_list():
        for ins in grp:
            e(ins)
    for ins in advance_k():
        e(ins)
    e(f"s_xor_b32 s{S_MBASE}, {STAGE}, s{S_MBASE}")     # back to stage 0 (refilled with step 2)
    e("s_waitcnt vmcnt(16)")
    e("s_barrier")
    for ins in frag_reads(SET0_A, SET0_B, V_RA, V_RB, 0):
        e(ins)
    if epi == "bias":
        # this tile's 8 bias values per lane (fp32): aux + col0 * 4 + lane offset
        e(f"s_lshl_b32 s{S_T0}, s{S_COL0}, 2")
        e(f"s_add_u32 s{S_SRDX}, s{S_AUX0}, s{S_T0}")
        e(f"s_addc_u32 s{S_SRDX + 1}, s{S_AUX0 + 1}, 0")
        e(f"s_mov_b32 s{S_SRDX + 2}, 1024")
        e(f"s_mov_b32 s{S_SRDX + 3}, 0x20000")
        e(f"buffer_load_dwordx4 {vr(V_BIAS)}, v{V_T + 1}, {sr(S_SRDX, 4)}, 0 offen")
        e(f"buffer_load_dwordx4 {vr(V_BIAS + 4)}, v{V_T + 1}, {sr(S_SRDX, 4)}, 0 offen offset:16")
    e("s_waitcnt lgkmcnt(0)")
    # K-steps: first, loop x (kt - 3), penult, last  (kt >= 4)
    iteration(e, "first")
    e(f"s_sub_u32 s{S_LOOP}, s{S_KT}, 3")
    e.label(e.L("kloop"))
    iteration(e, "loop")
    e(f"s_sub_u32 s{S_LOOP}, s{S_LOOP}, 1")
    e(f"s_cmp_eq_u32 s{S_LOOP}, 0")
    e("s_cbranch_scc0 " + e.L("kloop"))
    iteration(e, "penult")
    iteration(e, "last")
    # every wave's last LDS reads are retired (waited inside 'last'); the stages are free after this
    e("s_barrier")
    # reset the fragment bases to stage 0 for the next tile (kt is even: they toggled kt - 1 times)
    e(f"v_and_b32 v{V_RA}, 0xffff, v{V_RA}")
    e(f"v_and_b32 v{V_RB}, 0xffff, v{V_RB}")
    # ---- epilogue ----
    for _ in range(3):
        e("s_nop 7")
    if epi == "bias":
        e("s_waitcnt vmcnt(0)")
    rot = 0
    for i in range(8):
        for r in range(4):
            t = V_EPI + (rot % 4) * 12
            rot += 1
            for j in range(8):
                e(f"v_accvgpr_read_b32 v{t + j}, a{(i * 8 + j) * 4 + r}")
            if epi == "bias":
                for j in range(8):
                    e(f"v_add_f32 v{t + j}, v{t + j}, v{V_BIAS + j}")
            for p in range(4):
                e(f"v_cvt_pk_bf16_f32 v{t + 8 + p}, v{t + 2 * p}, v{t + 2 * p + 1}")
            e(f"s_mul_i32 s{S_SOFFC}, s{S_LDC2}, {16 * i + r}")
            e(f"buffer_store_dwordx4 {vr(t + 8)}, v{V_CO}, {sr(S_SRDC, 4)}, s{S_SOFFC} offen")
    e(f"s_add_u32 s{S_TILE}, s{S_TILE}, s{S_GRID}")
    e("s_branch " + e.L("tile"))
    e.label(e.L("end"))
    e("s_waitcnt vmcnt(0)")
    e("s_endpgm")
    return e.text()


def udiv(e, q, n, d, r):
    """s[q] = s[n] / s[d], s[r] = s[n] % s[d] for s[n] < 2^20, s[d] <= 2^12 (shift-subtract, 20 steps)"""
    e(f"s_mov_b32 s{q}, 0")
    e(f"s_mov_b32 s{r}, s{n}")
    for b in range(19, -1, -1):
        lab = e.fresh("div")
        e(f"s_lshl_b32 s{S_T3}, s{d}, {b}")
        e(f"s_cmp_ge_u32 s{r}, s{S_T3}")
        e(f"s_cbranch_scc0 {lab}")
        e(f"s_sub_u32 s{r}, s{r}, s{S_T3}")
        e(f"s_or_b32 s{q}, s{q}, {1 << b}")
        e.label(lab)


def set_srd(e, srd, ptr, row0, ld, nr):
    e(f"s_mul_i32 s{S_T0}, s{row0}, s{ld}")
    e(f"s_mul_hi_u32 s{S_T1}, s{row0}, s{ld}")
    e(f"s_lshl_b64 s[{S_T0}:{S_T1}], s[{S_T0}:{S_T1}], 1")
    e(f"s_add_u32 s{srd}, s{ptr}, s{S_T0}")
    e(f"s_addc_u32 s{srd + 1}, s{ptr + 1}, s{S_T1}")
    e(f"s_lshl_b32 s{nr}, s{ld}, 9")               # 256 rows * 2 bytes
    e(f"s_mov_b32 s{srd + 2}, s{nr}")
    e(f"s_mov_b32 s{srd + 3}, 0x20000")


KERNARG_SIZE = 96


def metadata(name):
    args = []
    off = 0
    for _ in range(6):
        args.append(f"""      - .address_space:  global
        .offset:         {off}
        .size:           8
        .value_kind:     global_buffer""")
        off += 8
    for _ in range(12):
        args.append(f"""      - .offset:         {off}
        .size:           4
        .value_kind:     by_value""")
        off += 4
    return f"""  - .agpr_count:     256
    .args:
{chr(10).join(args)}
    .group_segment_fixed_size: {2 * STAGE}
    .kernarg_segment_align: 8
    .kernarg_segment_size: {KERNARG_SIZE}
    .max_flat_workgroup_size: 256
    .name:           {name}
    .private_segment_fixed_size: 0
    .sgpr_count:     {S_LAST + 6}
    .sgpr_spill_count: 0
    .symbol:         {name}.kd
    .uniform_work_group_size: 1
    .uses_dynamic_stack: false
    .vgpr_count:     512
    .vgpr_spill_count: 0
    .wavefront_size: 64
"""


def descriptor(name):
    return f"""	.section	.rodata,"a",@progbits
	.p2align	6, 0x0
	.amdhsa_kernel {name}
		.amdhsa_group_segment_fixed_size {2 * STAGE}
		.amdhsa_private_segment_fixed_size 0
		.amdhsa_kernarg_size {KERNARG_SIZE}
		.amdhsa_user_sgpr_count 2
		.amdhsa_user_sgpr_kernarg_segment_ptr 1
		.amdhsa_system_sgpr_workgroup_id_x 1
		.amdhsa_system_vgpr_workitem_id 0
		.amdhsa_next_free_vgpr 512
		.amdhsa_next_free_sgpr {S_LAST}
		.amdhsa_accum_offset 256
		.amdhsa_reserve_vcc 1
		.amdhsa_float_denorm_mode_32 3
		.amdhsa_float_denorm_mode_16_64 3
		.amdhsa_dx10_clamp 1
		.amdhsa_ieee_mode 0
		.amdhsa_tg_split 0
	.end_amdhsa_kernel
	.text
"""


KERNELS = [("dalle_gemm_nt_plain", "plain"), ("dalle_gemm_nt_bias", "bias")]


def main(out):
    parts = ['\t.amdgcn_target "amdgcn-amd-amdhsa--gfx950"', "\t.amdhsa_code_object_version 6", "\t.text"]
    metas = []
    for name, epi in KERNELS:
        parts += [f"\t.globl\t{name}", "\t.p2align\t8", f"\t.type\t{name},@function", f"{name}:"]
        parts.append(kernel(name, epi))
        parts.append(f"\t.size\t{name}, .-{name}")
        parts.append(descriptor(name))
        metas.append(metadata(name))
    parts.append("\t.amdgpu_metadata\n---\namdhsa.kernels:\n" + "".join(metas)
                 + "amdhsa.target:   amdgcn-amd-amdhsa--gfx950\namdhsa.version:\n  - 1\n  - 2\n...\n\n\t.end_amdgpu_metadata")
    with open(out, "w") as f:
        f.write("\n".join(parts) + "\n")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gemm_gfx950.s")
