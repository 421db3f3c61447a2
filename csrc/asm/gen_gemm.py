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
* LDS: two 64 KB stages {A image 32 KB | B image 32 KB}.  An operand image is row-major, 256 rows x 128 B
  (the K-step's 64 bf16), and the 16-byte chunk c of image row r sits at position ``c ^ ((r >> 1) & 7)``.
  The LDS-DMA (``buffer_load_dwordx4 ... lds``: lane-linear 1 KB per instruction) fills 8 image rows x 128 B
  per instruction -- whole 128-byte global lines -- with the swizzle applied on the per-lane SOURCE address.
  A fragment (16 rows x 32 k) is one ``ds_read_b128`` per lane, bank-conflict free under the b128 lane
  grouping (checked in tests/test_asm_cpu.py).
* B image row ``16 f + c`` of a wave half holds global row ``8 c + f``: column fragment f then covers output
  columns ``8 c + f`` (c = lane & 15), so after the MFMAs each lane holds, for one output row, 8 CONSECUTIVE
  columns across its 8 column fragments; the epilogue writes 16 bytes per lane and 8 whole 128-byte lines
  per store instruction with no cross-lane exchange.
* Pipeline (per K-step t, stage X = t & 1): the k-half-1 fragments of step t are read into the second
  register set under the first 32 MFMAs (k-half 0 set); barrier B2 (everyone's reads of stage X retired)
  then the LDS-DMA of step t + 2 is issued INTO stage X under the next MFMAs (two steps ahead in two
  stages: a stage is refilled as soon as its last reads retire); ``vmcnt(16)`` + barrier B3 (step t + 1's
  DMA landed everywhere) and the k-half-0 fragments of step t + 1 are read from stage Y under the last 32
  MFMAs.  Two barriers per 128 MFMAs; no MFMA waits on a fragment read.
* Output mapping per lane l (c = l & 15, g = l >> 4), fragment (i, j), register r:
  ``C[row0 + 128 wm + 16 i + 4 g + r][col0 + 128 wn + 8 c + j]``.

Epilogues (``EPI``): ``plain`` (bf16 C), ``bias`` (bf16 C + fp32 bias[n]).
Diagnostic builds (``--diag``, measurement only, never loaded by the framework): ``noepi`` (no epilogue),
``nodma`` (main loop without its LDS-DMA; wrong results by design).

Usage:  gen_gemm.py OUT.s [--diag]     (assemble with clang -target amdgcn-amd-amdhsa -mcpu=gfx950)
"""
import re
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
S_OFFA = 36         # 8 soffsets of the A DMA instructions (s36..s43): 8 s rows
S_OFFB = 44         # 8 soffsets of the B DMA instructions (s44..s51): (s >> 1) rows
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
S_TM, S_TNI = 67, 68  # tile row / column index
# grouped tile order (8 tile rows per group, column-major inside a group): 8 * tiles_n, its division magic,
# tiles in full groups, first row of the partial group, its row count and division magic
S_G8, S_MAGG, S_FULL, S_TMFULL, S_ROWREM, S_MAGR = 69, 70, 71, 76, 77, 78
S_SRDX = 72         # s[72:75] a spare resource (epilogue operands)
S_KV, S_WRAP, S_S0B = 79, 80, 81   # K-slice of the next DMA, 128 - 2 K (the wrap step), first slice * 128
S_LAST = 100

# VGPRs
V_TID = 0
V_GA0, V_GA1, V_GB0, V_GB1 = 1, 2, 3, 4     # per-lane LDS-DMA source offsets (even / odd instruction s)
V_RA0, V_RA1, V_RB0, V_RB1 = 5, 6, 7, 8     # per-lane fragment read bases (k-half 0 / 1) in stage X
V_CO = 9                                     # per-lane epilogue C offset
V_T = 10                                     # temps v10, v11
V_BOFF = 12                                  # per-lane bias byte offset
SET0_A, SET0_B, SET1_A, SET1_B = 16, 48, 80, 112   # 4 fragment register blocks of 32 VGPRs
V_EPI = 144                                  # epilogue scratch (4 rotating sets of 12)
V_BIAS = 248                                 # 8 bias values per lane (v248..v255)

STAGE = 65536
B_IMG = 32768
PIECE = 1024
ROWB = 128          # bytes per operand image row (one K-step)


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
SERPENTINE = False   # (measurement build "serp": j reversed on odd i, so consecutive MFMAs at a row change share B)


def mfma_list(set_a, set_b, zero_c):
    """the 64 MFMAs of one k-half (i-major), as instruction strings"""
    out = []
    for i in range(8):
        for j in (range(7, -1, -1) if SERPENTINE and i & 1 else range(8)):
            c = "0" if zero_c else acc(i, j)
            out.append(f"v_mfma_f32_16x16x32_bf16 {acc(i, j)}, {vr(set_a + 4 * i)}, {vr(set_b + 4 * j)}, {c}")
    return out


READ_ORDER = [("A", 0)] + [("B", j) for j in range(8)] + [("A", i) for i in range(1, 8)]   # consumption order


def frag_reads(set_a, set_b, h):
    """16 ds_read_b128: the 8 A fragments and 8 B fragments of k-half h (fragment f = image rows 16 f..), in
    the order the i-major MFMAs consume them (A0, B0..B7, A1..A7) so that counted lgkmcnt waits release
    each MFMA as soon as its two operands are in"""
    if TN:
        return tn_frag_reads(set_a, set_b, h)
    ra, rb = (V_RA0, V_RB0) if h == 0 else (V_RA1, V_RB1)
    out = []
    for op, f in READ_ORDER:
        if op == "A":
            out.append(f"ds_read_b128 {vr(set_a + 4 * f)}, v{ra} offset:{f * 16 * ROWB}")
        else:
            out.append(f"ds_read_b128 {vr(set_b + 4 * f)}, v{rb} offset:{f * 16 * ROWB}")
    return out


def set0_waits(set1_slots):
    """{n: lgkmcnt} waits placed before MFMA n (n = 1..63) of a step whose k-half-0 fragments were the last 16
    LDS reads of the previous step (A0 / B0 waited there): MFMA n needs read index max(idx(A[n // 8]),
    idx(B[n % 8])); the k-half-1 reads issued in this step's slots before it are younger and may stay
    pending.  lgkmcnt holds 4 bits: counts above 15 are clamped (a stricter wait)."""
    idx = {k: n for n, k in enumerate(READ_ORDER)}
    waits, have = {}, idx[("B", 0)]
    for n in range(1, 64):
        need = max(idx[("A", n // 8)], idx[("B", n % 8)])
        if need > have:
            younger = sum(1 for sl in set1_slots if sl <= n - 1)
            waits[n] = min(15, 15 - need + younger)
            have = need
    return waits


LOAD_POLICY = ("", "")   # cache-policy modifiers of the A / B LDS-DMA loads (measurement builds "ant", "abnt": streaming)


def glds_list():
    """16 LDS-DMA instructions of one K-step as (M0 write, DMA) pairs: this wave's A image rows 64q + 8s .. +7,
    then its B image rows (s = 0..7); M0 = S_MBASE (+ B_IMG) + s KB.  The M0 write needs one wait state
    before its DMA: in a slot schedule it goes one MFMA ahead (the MFMA is the wait state, no s_nop)."""
    out = []
    par = (lambda s: (s >> 1) & 1) if TN else (lambda s: s & 1)   # which per-lane source offset
    for s in range(8):
        out.append((f"s_add_u32 m0, s{S_MBASE}, {s * PIECE}",
                    f"buffer_load_dwordx4 v{V_GA1 if par(s) else V_GA0}, {sr(S_SRDA, 4)}, s{S_OFFA + s} offen{LOAD_POLICY[0]} lds"))
    for s in range(8):
        out.append((f"s_add_u32 m0, s{S_MBASE}, {B_IMG + s * PIECE}",
                    f"buffer_load_dwordx4 v{V_GB1 if par(s) else V_GB0}, {sr(S_SRDB, 4)}, s{S_OFFB + s} offen{LOAD_POLICY[1]} lds"))
    return out[8:] + out[:8] if (BFIRST and not TN) or (TN and TN_BFIRST) else out


BFIRST = True       # B's k-half-1 fragments, image release and DMA ahead of A's (~1 % on every plain shape,
                    # profiles/r5_asm_gemm_bfirst.jsonl): B -- re-read by every column tile -- gets the longer lead


STAGGER = True      # per-XCD K start (the diagnostic nostagger build turns it off)


def advance_k():
    """move both operand resources one K-slice (128 bytes) forward; with the staggered start a tile walks its
    slices s0, s0 + 1, .., kt - 1, 0, .., s0 - 1, so past the last slice the resources step back by 2 K - 128"""
    if TN:
        # the K-step is 64 ROWS of the token-major operands
        return [f"s_add_u32 s{S_SRDA}, s{S_SRDA}, s{S_STEPA}", f"s_addc_u32 s{S_SRDA + 1}, s{S_SRDA + 1}, 0",
                f"s_add_u32 s{S_SRDB}, s{S_SRDB}, s{S_STEPB}", f"s_addc_u32 s{S_SRDB + 1}, s{S_SRDB + 1}, 0"]
    if not STAGGER:
        return [
            f"s_add_u32 s{S_SRDA}, s{S_SRDA}, 128", f"s_addc_u32 s{S_SRDA + 1}, s{S_SRDA + 1}, 0",
            f"s_sub_u32 s{S_NRA}, s{S_NRA}, 128", f"s_mov_b32 s{S_SRDA + 2}, s{S_NRA}",
            f"s_add_u32 s{S_SRDB}, s{S_SRDB}, 128", f"s_addc_u32 s{S_SRDB + 1}, s{S_SRDB + 1}, 0",
            f"s_sub_u32 s{S_NRB}, s{S_NRB}, 128", f"s_mov_b32 s{S_SRDB + 2}, s{S_NRB}",
        ]
    return [
        f"s_add_u32 s{S_KV}, s{S_KV}, 1",
        f"s_cmp_eq_u32 s{S_KV}, s{S_KT}",
        f"s_cselect_b32 s{S_T2}, s{S_WRAP}, 128",       # byte step (low word)
        f"s_cselect_b32 s{S_T3}, -1, 0",                 # its sign extension
        f"s_cselect_b32 s{S_KV}, 0, s{S_KV}",
        f"s_add_u32 s{S_SRDA}, s{S_SRDA}, s{S_T2}", f"s_addc_u32 s{S_SRDA + 1}, s{S_SRDA + 1}, s{S_T3}",
        f"s_sub_u32 s{S_NRA}, s{S_NRA}, s{S_T2}", f"s_mov_b32 s{S_SRDA + 2}, s{S_NRA}",
        f"s_add_u32 s{S_SRDB}, s{S_SRDB}, s{S_T2}", f"s_addc_u32 s{S_SRDB + 1}, s{S_SRDB + 1}, s{S_T3}",
        f"s_sub_u32 s{S_NRB}, s{S_NRB}, s{S_T2}", f"s_mov_b32 s{S_SRDB + 2}, s{S_NRB}",
    ]


def stagger_setup(e):
    """first K-slice of every tile of this workgroup: (XCD) * (kt / 8) -- the 8 XCDs stream different K
    columns of A / B at any moment (no channel hot spot at long row pitches) while the 32 CUs of one XCD
    keep walking the same slices (their shared panels stay L2 hits)"""
    if STAGGER:
        e(f"s_and_b32 s{S_T0}, s{S_WG}, 7")
        e(f"s_lshr_b32 s{S_T1}, s{S_KT}, 3")
        e(f"s_mul_i32 s{S_T0}, s{S_T0}, s{S_T1}")
        e(f"s_lshl_b32 s{S_S0B}, s{S_T0}, 7")
    else:
        e(f"s_mov_b32 s{S_S0B}, 0")
    e(f"s_lshl_b32 s{S_T0}, s{S_K}, 1")
    e(f"s_sub_u32 s{S_WRAP}, 128, s{S_T0}")


def toggle_reads():
    """the fragment read bases move to the other stage (at B3: the next step's data)"""
    regs = list(range(V_TRA, V_TRA + 4)) + list(range(V_TRB, V_TRB + 4)) if TN else (V_RA0, V_RA1, V_RB0, V_RB1)
    return [f"v_xor_b32 v{v}, {STAGE}, v{v}" for v in regs]


# slot map of one K-step (instructions issued after MFMA n, n = 0..127), measured on the B128 shapes
# (profiles/r5_asm_gemm_diag.txt): the LDS-DMA costs issue time roughly per instruction unless spread out
# (16 DMAs every 3 MFMAs: 1402 TF at K = 8192; packed one per MFMA: 1298; every ~5.6: +8 %), while waiting
# for it to land costs nothing measurable (no-wait variant: +0.6 %) -- so the DMA is spread over the whole
# step after B2 and B3 sits in the middle of it.
B2_SLOT = 36
B3_SLOT = 90
DMA_SLOTS = [40 + round(5.6 * n) for n in range(16)]          # 40 .. 124
PLAIN_B2, PLAIN_DMA = B2_SLOT, DMA_SLOTS   # (measurement builds "b2_33": release at 33, DMA 35..123; "dma_dense": DMA 38..98)
PLAIN_SCHEDS = {"b2_33": (33, [35 + round(5.9 * n) for n in range(16)]), "dma_dense": (36, [38 + 4 * n for n in range(16)])}
ADVANCE_SLOT = 126
# split release (default): the k-half-1 A fragments are read first and a barrier (BA) frees the stage's A image
# early, so its 8 DMAs start under MFMA 20 while the B fragments are still being read; a second barrier (BB)
# frees the B image for the other 8.  16 DMAs over MFMAs 20..124 instead of 40..124.
SPLIT = True
SPLIT_SET1_SLOTS = [2 * n for n in range(8)] + [22 + 3 * n for n in range(8)]   # A0..A7, then B0..B7
BA_SLOT, BB_SLOT = 18, 46
SPLIT_DMA_SLOTS = [20 + 4 * n for n in range(8)] + [54 + 10 * n for n in range(8)]   # 20 .. 48, 54 .. 124


STORE_SLOTS = [3 + 4 * n for n in range(8)]                   # deferred epilogue stores: before B2


def iteration(e, kind, diag=None, extra=0, prefetch=False, pre=(), stores=(), head=(), work=(), work_span=(40, 120),
              work2=(), work2_span=(60, 118), at=(), more=()):
    """one K-step.  kind: 'first' (zero-init accumulators, DMA t+2), 'loop' (DMA t+2),
    'penult' (no DMA of this tile, wait all), 'last' (no DMA of this tile, no next reads).
    ``prefetch`` (penult / last of a tile that has a successor): the stage freed at B2 receives the NEXT
    tile's K-step 0 (penult) / 1 (last), so that tile starts with both stages loaded and the DMA issue hides
    under these steps' MFMAs. ``pre``: scalar instructions spread in order over MFMAs 1..33 (next-tile setup).
    ``stores``: instruction groups (the previous tile's deferred epilogue stores) issued early in the step,
    older than this step's DMA; ``extra``: VMEM operations issued after the previous step's DMA and before
    this step's B3 that B3 need not wait for (issued by the caller between the previous step and this one;
    every VMEM instruction this step places before B3 is counted here).  ``head``: instructions before MFMA 0;
    ``work``: instructions spread in order over the MFMA gaps of ``work_span`` (a fused epilogue's deferred
    work; its VMEM must sit before the step's last DMA); ``work2`` / ``more`` ((list, span) pairs): the same;
    ``at``: (slot, instruction) pairs placed exactly.
    Returns this step's VMEM instructions in issue order.
    Entry: SET0 holds this step's k-half-0 fragments (waited); the read bases point at stage X."""
    m0 = mfma_list(SET0_A, SET0_B, kind == "first")
    m1 = mfma_list(SET1_A, SET1_B, False)
    slots = [[] for _ in range(128)]  # instructions issued after MFMA n
    # k-half-1 fragments of this step (stage X) under MFMAs 0..31 (0..43 split: all A first)
    if TN:
        set1_slots = TN_SET1_SLOTS
        reads = frag_reads(SET1_A, SET1_B, 1)      # 16 A then 16 B transposed reads
        if TN_BFIRST:
            reads = reads[16:] + reads[:16]
        dma_slots = TN_ONEBAR_DMA_SLOTS if TN_ONEBAR else TN_DMA_SLOTS
    elif SPLIT:
        set1_slots = SPLIT_SET1_SLOTS
        reads = frag_reads(SET1_A, SET1_B, 1)
        ra_ = [r for r in reads if f", v{V_RA1} " in r]
        rb_ = [r for r in reads if f", v{V_RB1} " in r]
        reads = rb_ + ra_ if BFIRST else ra_ + rb_
        assert len(reads) == 16
        dma_slots = SPLIT_DMA_SLOTS
    else:
        set1_slots = [2 * n for n in range(16)]
        reads = frag_reads(SET1_A, SET1_B, 1)
        dma_slots = PLAIN_DMA
    for n, ins in zip(set1_slots, reads):
        slots[n].append(ins)
    # the k-half-0 fragments still in flight from the previous step: wait for each as its MFMA comes up
    if not TN:
        for n, cnt in set0_waits(sorted(set1_slots)).items():
            slots[n - 1].append(f"s_waitcnt lgkmcnt({cnt})")
    # pre: before the first M0 write (an SALU add: it rewrites SCC, which the pre sequences use)
    pre_end = BA_SLOT if SPLIT else 34
    for n, ins in enumerate(pre):
        slots[1 + n * (pre_end - 1) // len(pre)].append(ins)
    assert len(stores) <= len(STORE_SLOTS)
    for n, grp in enumerate(stores):
        slots[STORE_SLOTS[n]].extend(grp)
    for wk, (lo, hi) in ((work, work_span), (work2, work2_span)) + tuple(more):
        if wk:
            assert hi <= 120
            for n, ins in enumerate(wk):
                slots[lo + n * (hi - lo) // len(wk)].append(ins)
    for n, ins in at:
        slots[n].append(ins)
    dma = (kind in ("first", "loop") or prefetch) and diag != "nodma"
    if dma and (SPLIT or TN) and not (TN and TN_ONEBAR):
        # BA after the A k-half-1 reads (and this step's k-half-0 reads) retired: stage X's A image is free;
        # BB after the B reads: its B image.  Each refilled with step t + 2's piece.
        ba, bb = (TN_BA_SLOT, TN_BB_SLOT) if TN else (BA_SLOT, BB_SLOT)
        # BA waits for the A reads only: the B reads issued since are younger (LDS returns in order)
        n_b = sum(1 for sl in set1_slots[len(set1_slots) // 2:] if sl <= ba)
        slots[ba].append(f"s_waitcnt lgkmcnt({n_b})")
        slots[ba].append("s_barrier")
        slots[bb].append("s_waitcnt lgkmcnt(0)")
        slots[bb].append("s_barrier")
    elif dma:
        # B2 after the k-half-1 reads retired: stage X is free; refill it with step t + 2
        b2 = TN_B2_SLOT if TN else PLAIN_B2
        slots[b2].append("s_waitcnt lgkmcnt(0)")
        slots[b2].append("s_barrier")
    else:
        slots[max(set1_slots) + 2].append("s_waitcnt lgkmcnt(0)")
    if dma:
        for n, (m0w, ins) in enumerate(glds_list()):
            slots[dma_slots[n] - 1].append(m0w)
            slots[dma_slots[n]].append(ins)
    if dma or kind in ("first", "loop"):
        # after this step's last DMA: the resources move one K-step and the DMA base to the other stage
        slots[ADVANCE_SLOT].extend(advance_k() + [f"s_xor_b32 s{S_MBASE}, {STAGE}, s{S_MBASE}"])
    if kind != "last":
        # B3: step t + 1's DMA (issued during the previous step) landed for every wave; the DMA of this
        # step issued so far may stay in flight. Then read step t + 1's k-half-0 fragments from stage Y.
        younger = sum(1 for n in range(B3_SLOT + 1) for ins in slots[n] if ins.startswith("buffer_")) + extra
        assert younger < 64
        slots[B3_SLOT].append(f"s_waitcnt vmcnt({younger})")
        slots[B3_SLOT].append("s_barrier")
        slots[B3_SLOT].extend(toggle_reads())
        busy = set(dma_slots) if dma else set()
        free = [n for n in range(B3_SLOT + 2, 126 if TN else 124) if n not in busy]
        reads0 = frag_reads(SET0_A, SET0_B, 0)
        pick = [free[round(i * (len(free) - 1) / (len(reads0) - 1))] for i in range(len(reads0))]
        for n, ins in zip(pick, reads0):
            slots[n].append(ins)
        # MFMA 0 of the next step needs A0 / B0 (the first two of these 16 reads)
        slots[127].append("s_waitcnt lgkmcnt(0)" if TN else f"s_waitcnt lgkmcnt({16 - 2})")
    # deferred-work markers "@vmwait:TAG": wait until the VMEM instruction(s) tagged "; @TAG" (placed
    # earlier in this step) have completed -- vmcnt(number of VMEM instructions issued after the last one);
    # "@vmwait_prev:K": until a VMEM instruction of an EARLIER step followed by K others there has completed
    order = [(n, k) for n in range(128) for k in range(len(slots[n]))]
    vm_seen = []
    for n, k in order:
        ins = slots[n][k]
        if ins.startswith("@vmwait_prev:"):
            cnt = int(ins.split(":", 1)[1]) + len(vm_seen)
            assert cnt < 64
            slots[n][k] = f"s_waitcnt vmcnt({cnt})"
        elif ins.startswith("@vmwait:"):
            tag = ins.split(":", 1)[1]
            tagged = [i for i, x in enumerate(vm_seen) if x.endswith("; @" + tag)]
            assert tagged or GB_DIAG == "nomem", f"no VMEM tagged {tag} before its wait"
            slots[n][k] = f"s_waitcnt vmcnt({len(vm_seen) - 1 - max(tagged)})" if tagged else "s_nop 0"
        elif ins.startswith("buffer_"):
            vm_seen.append(ins)
    mf = m0 + m1
    for ins in head:
        e(ins)
    for n in range(128):
        e(mf[n])
        for ins in slots[n]:
            e(ins)
    return [ins for n in range(128) for ins in slots[n] if ins.startswith("buffer_")]


# ----------------------------------------------------------------------------------------------------
# kernel
# ----------------------------------------------------------------------------------------------------
def lane_setup(e, epi, diag=None):
    """per-lane offsets (DMA sources, fragment read bases, epilogue) from the wave id and lane"""
    T0, T1 = V_T, V_T + 1
    # ---- fragment read bases: wave image half + lane row (p = lane & 15) + swizzled chunk (kg = lane >> 4) ----
    #   k-half h: row p, chunk 4 h + kg at position (4 h + kg) ^ ((p >> 1) & 7)
    e(f"v_and_b32 v{T0}, 15, v{V_TID}")                  # p
    e(f"v_lshrrev_b32 v{T1}, 1, v{T0}")                  # p >> 1 (< 8)
    e(f"v_lshrrev_b32 v{V_RA0}, 4, v{V_TID}")
    e(f"v_and_b32 v{V_RA0}, 3, v{V_RA0}")                 # kg
    e(f"v_xor_b32 v{V_RA1}, 4, v{V_RA0}")                 # 4 + kg
    e(f"v_xor_b32 v{V_RA0}, v{V_RA0}, v{T1}")
    e(f"v_xor_b32 v{V_RA1}, v{V_RA1}, v{T1}")
    e(f"v_lshlrev_b32 v{V_RA0}, 4, v{V_RA0}")
    e(f"v_lshlrev_b32 v{V_RA1}, 4, v{V_RA1}")
    e(f"v_lshl_add_u32 v{V_RA0}, v{T0}, 7, v{V_RA0}")     # + p * 128
    e(f"v_lshl_add_u32 v{V_RA1}, v{T0}, 7, v{V_RA1}")
    e(f"v_add_u32 v{V_RB0}, {B_IMG}, v{V_RA0}")
    e(f"v_add_u32 v{V_RB1}, {B_IMG}, v{V_RA1}")
    e(f"s_lshr_b32 s{S_T0}, s{S_WAVE}, 1")
    e(f"s_lshl_b32 s{S_T0}, s{S_T0}, 14")                # wm * 16 KB
    e(f"s_and_b32 s{S_T1}, s{S_WAVE}, 1")
    e(f"s_lshl_b32 s{S_T1}, s{S_T1}, 14")                # wn * 16 KB
    e(f"v_add_u32 v{V_RA0}, s{S_T0}, v{V_RA0}")
    e(f"v_add_u32 v{V_RA1}, s{S_T0}, v{V_RA1}")
    e(f"v_add_u32 v{V_RB0}, s{S_T1}, v{V_RB0}")
    e(f"v_add_u32 v{V_RB1}, s{S_T1}, v{V_RB1}")
    # ---- DMA sources: lane t -> image row r' = t >> 3 of the instruction, position c' = t & 7,
    #      global chunk c' ^ (4 (s & 1) + (r' >> 1)) ----
    e(f"v_lshrrev_b32 v{T0}, 3, v{V_TID}")
    e(f"v_and_b32 v{T0}, 7, v{T0}")                      # r'
    e(f"v_and_b32 v{T1}, 7, v{V_TID}")                   # c'
    e(f"v_lshrrev_b32 v{V_GB0}, 1, v{T0}")
    e(f"v_xor_b32 v{V_GA0}, v{T1}, v{V_GB0}")            # c' ^ (r' >> 1)
    e(f"v_xor_b32 v{V_GA1}, 4, v{V_GA0}")                # c' ^ (4 + (r' >> 1))
    e(f"v_lshlrev_b32 v{V_GA0}, 4, v{V_GA0}")
    e(f"v_lshlrev_b32 v{V_GA1}, 4, v{V_GA1}")
    e(f"v_mov_b32 v{V_GB0}, v{V_GA0}")
    e(f"v_mov_b32 v{V_GB1}, v{V_GA1}")
    # A row: 64 q + r'
    e(f"s_lshl_b32 s{S_T0}, s{S_WAVE}, 6")
    e(f"v_add_u32 v{T1}, s{S_T0}, v{T0}")
    e(f"s_lshl_b32 s{S_T2}, s{S_LDA}, 1")                # lda * 2
    e(f"v_mad_u32_u24 v{V_GA0}, v{T1}, s{S_T2}, v{V_GA0}")
    e(f"v_mad_u32_u24 v{V_GA1}, v{T1}, s{S_T2}, v{V_GA1}")
    # B row: 128 (q >> 1) + 4 (q & 1) + 8 r' (+ 64 for odd s)
    e(f"s_lshr_b32 s{S_T0}, s{S_WAVE}, 1")
    e(f"s_lshl_b32 s{S_T0}, s{S_T0}, 7")
    e(f"s_and_b32 s{S_T1}, s{S_WAVE}, 1")
    e(f"s_lshl_b32 s{S_T1}, s{S_T1}, 2")
    e(f"s_add_u32 s{S_T0}, s{S_T0}, s{S_T1}")
    e(f"v_lshl_add_u32 v{T1}, v{T0}, 3, s{S_T0}")
    e(f"s_lshl_b32 s{S_T3}, s{S_LDB}, 1")                # ldb * 2
    e(f"v_mad_u32_u24 v{V_GB0}, v{T1}, s{S_T3}, v{V_GB0}")
    e(f"v_add_u32 v{T1}, 64, v{T1}")
    e(f"v_mad_u32_u24 v{V_GB1}, v{T1}, s{S_T3}, v{V_GB1}")
    # instruction soffsets: A 8 s rows, B (s >> 1) rows
    for s in range(8):
        e(f"s_mul_i32 s{S_OFFA + s}, s{S_T2}, {8 * s}")
        e(f"s_mul_i32 s{S_OFFB + s}, s{S_T3}, {s >> 1}")
    # ---- epilogue offset: row 128 wm + 4 g, col 128 wn + 8 c (bytes, relative to the tile) ----
    e(f"v_lshrrev_b32 v{T0}, 4, v{V_TID}")
    e(f"v_and_b32 v{T0}, 3, v{T0}")
    e(f"v_lshlrev_b32 v{T0}, 2, v{T0}")                  # 4 g
    e(f"s_lshr_b32 s{S_T0}, s{S_WAVE}, 1")
    e(f"s_lshl_b32 s{S_T0}, s{S_T0}, 7")
    e(f"v_add_u32 v{T0}, s{S_T0}, v{T0}")                # row
    e(f"v_mul_lo_u32 v{V_CO}, v{T0}, s{S_LDC2}")
    e(f"v_and_b32 v{T0}, 15, v{V_TID}")
    e(f"v_lshlrev_b32 v{T0}, 4, v{T0}")                  # 8 c columns * 2 bytes
    e(f"s_and_b32 s{S_T1}, s{S_WAVE}, 1")
    e(f"s_lshl_b32 s{S_T1}, s{S_T1}, 8")                # 128 wn * 2 bytes
    e(f"v_add_u32 v{T0}, s{S_T1}, v{T0}")
    e(f"v_add_u32 v{V_CO}, v{V_CO}, v{T0}")
    if epi == "bias":
        # byte offset of this lane's 8 bias values relative to col0: (128 wn + 8 c) * 4
        e(f"v_and_b32 v{V_BOFF}, 15, v{V_TID}")
        e(f"v_lshlrev_b32 v{V_BOFF}, 5, v{V_BOFF}")
        e(f"s_and_b32 s{S_T1}, s{S_WAVE}, 1")
        e(f"s_lshl_b32 s{S_T1}, s{S_T1}, 9")
        e(f"v_add_u32 v{V_BOFF}, s{S_T1}, v{V_BOFF}")


def setup_operands(e):
    """row0 / col0 of tile (S_TM, S_TNI), the A / B resources at the tile's panels, DMA base at stage 0"""
    e(f"s_lshl_b32 s{S_ROW0}, s{S_TM}, 8")
    e(f"s_lshl_b32 s{S_COL0}, s{S_TNI}, 8")
    set_srd(e, S_SRDA, S_A, S_ROW0, S_LDA, S_NRA)
    set_srd(e, S_SRDB, S_B, S_COL0, S_LDB, S_NRB)
    if STAGGER:
        for srd, nr in ((S_SRDA, S_NRA), (S_SRDB, S_NRB)):
            e(f"s_add_u32 s{srd}, s{srd}, s{S_S0B}")
            e(f"s_addc_u32 s{srd + 1}, s{srd + 1}, 0")
            e(f"s_sub_u32 s{nr}, s{nr}, s{S_S0B}")
            e(f"s_mov_b32 s{srd + 2}, s{nr}")
        e(f"s_lshr_b32 s{S_KV}, s{S_S0B}, 7")
    e(f"s_lshl_b32 s{S_MBASE}, s{S_WAVE}, 13")  # stage-0 DMA base of this wave's pieces: q * 8 KB


def tile_coords():
    """(S_TM, S_TNI) of tile S_TILE in the grouped order: tile rows in groups of 8, column-major inside a
    group, so the 32 tiles an XCD takes per round (consecutive ids) form an 8 x 4 block -- 8 A panels and 4 B
    panels in its L2 instead of 1 A panel and 32 B panels (the row-major order at tiles_n = 32).  The partial
    last group (tile rows % 8 rows) is column-major over its own rows.  Divisions are multiply-high by
    ceil(2^32 / d) (exact for ids < 2^20, d < 2^12).  Branch-free SALU (spread over MFMA gaps)."""
    return [f"s_mul_hi_u32 s{S_T0}, s{S_TILE}, s{S_MAGG}",          # group
            f"s_mul_i32 s{S_T1}, s{S_T0}, s{S_G8}",
            f"s_sub_u32 s{S_T1}, s{S_TILE}, s{S_T1}",                # id inside the group
            f"s_and_b32 s{S_T2}, s{S_T1}, 7",
            f"s_lshl_b32 s{S_T0}, s{S_T0}, 3",
            f"s_add_u32 s{S_TM}, s{S_T0}, s{S_T2}",
            f"s_lshr_b32 s{S_TNI}, s{S_T1}, 3",
            f"s_sub_u32 s{S_T1}, s{S_TILE}, s{S_FULL}",              # id inside the partial group
            f"s_mul_hi_u32 s{S_T0}, s{S_T1}, s{S_MAGR}",
            f"s_cmp_eq_u32 s{S_MAGR}, 0",                            # one row: column = id
            f"s_cselect_b32 s{S_T0}, s{S_T1}, s{S_T0}",
            f"s_mul_i32 s{S_T2}, s{S_T0}, s{S_ROWREM}",
            f"s_sub_u32 s{S_T2}, s{S_T1}, s{S_T2}",
            f"s_add_u32 s{S_T2}, s{S_T2}, s{S_TMFULL}",
            f"s_cmp_ge_u32 s{S_TILE}, s{S_FULL}",
            f"s_cselect_b32 s{S_TM}, s{S_T2}, s{S_TM}",
            f"s_cselect_b32 s{S_TNI}, s{S_T0}, s{S_TNI}"]


def next_tile():
    return [f"s_add_u32 s{S_TILE}, s{S_TILE}, s{S_GRID}"] + tile_coords()


def tile_order_setup(e):
    """the constants of tile_coords (once per kernel)"""
    e(f"s_lshl_b32 s{S_G8}, s{S_TN}, 3")
    magic(e, S_MAGG, S_G8)
    e(f"s_lshr_b32 s{S_T3}, s{S_M}, 8")                    # tile rows
    e(f"s_and_b32 s{S_ROWREM}, s{S_T3}, 7")
    e(f"s_andn2_b32 s{S_TMFULL}, s{S_T3}, 7")
    e(f"s_mul_i32 s{S_FULL}, s{S_TMFULL}, s{S_TN}")
    magic(e, S_MAGR, S_ROWREM)
    e(f"s_cmp_lt_u32 s{S_ROWREM}, 2")
    e(f"s_cselect_b32 s{S_MAGR}, 0, s{S_MAGR}")


def magic(e, q, d):
    """s[q] = ceil(2^32 / s[d]) = floor((2^32 - 1) / s[d]) + 1 for 2 <= s[d] < 2^16 (restoring division)"""
    e(f"s_mov_b32 s{q}, 0")
    e(f"s_mov_b32 s{S_T1}, 0")
    for b in range(31, -1, -1):
        lab = e.fresh("mag")
        e(f"s_lshl_b32 s{S_T1}, s{S_T1}, 1")
        e(f"s_or_b32 s{S_T1}, s{S_T1}, 1")
        e(f"s_cmp_ge_u32 s{S_T1}, s{d}")
        e(f"s_cbranch_scc0 {lab}")
        e(f"s_sub_u32 s{S_T1}, s{S_T1}, s{d}")
        e(f"s_or_b32 s{q}, s{q}, {hex(1 << b)}")
        e.label(lab)
    e(f"s_add_u32 s{q}, s{q}, 1")


def emit_all(e, ins):
    for i in ins:
        e(i)


def setup_output(e):
    """C resource of the tile at (S_ROW0, S_COL0): base = C + (row0 * ldc + col0) * 2, 256 rows"""
    e(f"s_mul_i32 s{S_T0}, s{S_ROW0}, s{S_LDC}")
    e(f"s_mul_hi_u32 s{S_T1}, s{S_ROW0}, s{S_LDC}")
    e(f"s_add_u32 s{S_T0}, s{S_T0}, s{S_COL0}")
    e(f"s_addc_u32 s{S_T1}, s{S_T1}, 0")
    e(f"s_lshl_b64 s[{S_T0}:{S_T1}], s[{S_T0}:{S_T1}], 1")
    e(f"s_add_u32 s{S_SRDC}, s{S_C}, s{S_T0}")
    e(f"s_addc_u32 s{S_SRDC + 1}, s{S_C + 1}, s{S_T1}")
    e(f"s_lshl_b32 s{S_SRDC + 2}, s{S_LDC2}, 8")
    e(f"s_mov_b32 s{S_SRDC + 3}, 0x20000")


def prologue_dma(e):
    """K-steps 0 and 1 of the tile into stages 0 and 1 (32 DMA instructions per wave)"""
    for _ in range(2):
        for m0, dma in glds_list():
            e(m0)
            e("s_nop 0")
            e(dma)
        for ins in advance_k():
            e(ins)
        e(f"s_xor_b32 s{S_MBASE}, {STAGE}, s{S_MBASE}")
    # S_MBASE is back at stage 0 (refilled with step 2)


def body_head(e, epi, older_stores):
    """step 0's fragments and the tile's epilogue operands, then the first K-step. ``older_stores``: the
    previous tile's epilogue stores issued after this tile's DMA prologue (they count in vmcnt)."""
    for ins in frag_reads(SET0_A, SET0_B, 0):
        e(ins)
    nb = 0
    if epi == "bias":
        # this tile's 8 bias values per lane (fp32): aux + col0 * 4 + lane offset
        e(f"s_lshl_b32 s{S_T0}, s{S_COL0}, 2")
        e(f"s_add_u32 s{S_SRDX}, s{S_AUX0}, s{S_T0}")
        e(f"s_addc_u32 s{S_SRDX + 1}, s{S_AUX0 + 1}, 0")
        e(f"s_mov_b32 s{S_SRDX + 2}, 1024")
        e(f"s_mov_b32 s{S_SRDX + 3}, 0x20000")
        e(f"buffer_load_dwordx4 {vr(V_BIAS)}, v{V_BOFF}, {sr(S_SRDX, 4)}, 0 offen")
        e(f"buffer_load_dwordx4 {vr(V_BIAS + 4)}, v{V_BOFF}, {sr(S_SRDX, 4)}, 0 offen offset:16")
        nb = 2
    e("s_waitcnt lgkmcnt(0)")
    return older_stores + nb


def kernel(name, epi, diag=None):
    global STORE_POLICY, STAGGER, SPLIT, PLAIN_DIAG
    PLAIN_DIAG = diag if diag in ("nostore", "nopack") else None
    global BFIRST, SERPENTINE, LOAD_POLICY
    BFIRST = diag != "afirst"
    SERPENTINE = diag == "serp"
    LOAD_POLICY = {"ant": (" nt", ""), "abnt": (" nt", " nt")}.get(diag, ("", ""))
    global PLAIN_B2, PLAIN_DMA
    PLAIN_B2, PLAIN_DMA = PLAIN_SCHEDS.get(diag, (B2_SLOT, DMA_SLOTS))
    STORE_POLICY = "" if diag == "l2store" else " nt"
    STAGGER = diag != "nostagger"
    # plain / bias: one stage-release barrier (B2) -- 0.6-0.7 % faster than the split release on every plain
    # shape in a sustained (power-limited) A/B, profiles/r5_ab_sustained.txt; the fused kernels keep SPLIT
    SPLIT = diag == "split"
    e = Emitter(name)
    # ---- arguments ----
    e(f"s_load_dwordx8 {sr(S_A, 8)}, s[0:1], 0x0")          # A B C AUX0
    e(f"s_load_dwordx8 {sr(S_M, 8)}, s[0:1], 0x30")         # M N K lda ldb ldc tiles_n num_tiles
    e(f"s_load_dword s{S_GRID}, s[0:1], 0x50")
    e(f"v_lshrrev_b32 v{V_T}, 6, v{V_TID}")
    e("s_nop 1")   # VALU write -> v_readfirstlane of the same VGPR: gfx950 needs a wait state (hipcc pads it too)
    e(f"v_readfirstlane_b32 s{S_WAVE}, v{V_T}")
    e("s_nop 1")
    e("s_waitcnt lgkmcnt(0)")
    e(f"s_lshr_b32 s{S_KT}, s{S_K}, 6")
    e(f"s_lshl_b32 s{S_LDC2}, s{S_LDC}, 1")
    # the K-step schedule needs an even number of at least 4 steps (first, loop >= 1, penult, last; the next
    # tile's prefetch lands in stage 0 / 1): never run on anything else (the host rejects those shapes too)
    e(f"s_cmp_lt_u32 s{S_KT}, 4")
    e("s_cbranch_scc1 " + e.L("end"))
    e(f"s_bitcmp1_b32 s{S_KT}, 0")
    e("s_cbranch_scc1 " + e.L("end"))
    lane_setup(e, epi, diag)
    # ---- persistent tiles: tile = round * grid + (wg % 8) * (grid / 8) + wg / 8 ----
    e(f"s_and_b32 s{S_T0}, s{S_WG}, 7")
    e(f"s_lshr_b32 s{S_T1}, s{S_GRID}, 3")
    e(f"s_mul_i32 s{S_T0}, s{S_T0}, s{S_T1}")
    e(f"s_lshr_b32 s{S_T1}, s{S_WG}, 3")
    e(f"s_add_u32 s{S_TILE}, s{S_T0}, s{S_T1}")
    e(f"s_cmp_lt_u32 s{S_TILE}, s{S_NT}")
    e("s_cbranch_scc0 " + e.L("end"))
    tile_order_setup(e)
    stagger_setup(e)
    emit_all(e, tile_coords())
    setup_operands(e)
    prologue_dma(e)
    e("s_waitcnt vmcnt(16)")                    # step 0 landed (this wave's part) ...
    e("s_barrier")                              # ... and every wave's
    # first tile of the workgroup: nothing older than its DMA prologue
    extra = body_head(e, epi, 0)
    iteration(e, "first", diag, extra)
    e(f"s_sub_u32 s{S_LOOP}, s{S_KT}, 3")
    # K-steps: first, loop x (kt - 3), penult, last  (kt >= 4, even)
    e.label(e.L("kloop"))
    iteration(e, "loop", diag)
    e(f"s_sub_u32 s{S_LOOP}, s{S_LOOP}, 1")
    e(f"s_cmp_eq_u32 s{S_LOOP}, 0")
    e("s_cbranch_scc0 " + e.L("kloop"))
    e.label(e.L("tail"))
    # the last two K-steps.  The C resource of this tile is set in penult's first MFMA gaps (the previous
    # tile's deferred stores went out in steps 0..3); with a successor tile, the next_tile / operand setup
    # follow it there and these two steps DMA the successor's steps 0 and 1
    out = Emitter(e.prefix)
    setup_output(out)
    pre_out = [l.strip() for l in out.lines]
    sub = Emitter(e.prefix)
    setup_operands(sub)
    pre_next = pre_out + next_tile() + [l.strip() for l in sub.lines]
    e(f"s_add_u32 s{S_T0}, s{S_TILE}, s{S_GRID}")
    e(f"s_cmp_lt_u32 s{S_T0}, s{S_NT}")
    e("s_cbranch_scc0 " + e.L("final"))
    # ---- successor with deferred stores: 6 stores now, 26 packed into v[144:247] and issued under the
    #      successor's first K-steps (the HBM write of a tile overlaps the next tile's MFMAs instead of all CUs
    #      storing 128 KB at once): two per step over steps 0..12 when the tile has >= 16 K-steps (measured
    #      -1.5 % at N = 4096, -6 % at N = K = 1024 against [7, 7, 6, 6] over steps 0..3), else over 0..3 ----
    def deferred(defer):
        iteration(e, "penult", diag, prefetch=True, pre=pre_next)
        iteration(e, "last", diag, prefetch=True)
        tile_boundary(e)
        groups = epilogue_stash(e, epi) if diag != "noepi" else []
        n_imm = N_IMMEDIATE if groups and PLAIN_DIAG != "nostore" else 0
        e(f"s_waitcnt vmcnt({16 + n_imm})")         # the successor's step 0 landed (step 1 + the stores younger)
        e("s_barrier")
        extra = body_head(e, epi, n_imm)
        k = 0
        for n, cnt in enumerate(defer):
            grp = groups[k:k + cnt] if groups else []
            k += cnt
            iteration(e, "first" if n == 0 else "loop", diag, extra if n == 0 else 0, stores=grp)
        e(f"s_sub_u32 s{S_LOOP}, s{S_KT}, {3 + len(defer) - 1}")
        e(f"s_cmp_eq_u32 s{S_LOOP}, 0")
        e("s_cbranch_scc1 " + e.L("tail"))
        e("s_branch " + e.L("kloop"))

    if diag != "defer4":
        e(f"s_cmp_lt_u32 s{S_KT}, {3 + len(DEFER_LONG) - 1}")
        e("s_cbranch_scc1 " + e.L("defer4"))
        deferred(DEFER_LONG)
    e.label(e.L("defer4"))
    e(f"s_cmp_lt_u32 s{S_KT}, {3 + len(DEFER_SPLIT) - 1}")   # steps 0..3 peeled, penult after them
    e("s_cbranch_scc1 " + e.L("tail_imm"))
    deferred(DEFER_SPLIT)
    # ---- successor, 4 K-steps per tile: all 32 stores at the boundary ----
    e.label(e.L("tail_imm"))
    iteration(e, "penult", diag, prefetch=True, pre=pre_next)
    iteration(e, "last", diag, prefetch=True)
    tile_boundary(e)
    if diag != "noepi":
        epilogue_store(e, epi)
    n_all = 32 if diag != "noepi" and PLAIN_DIAG != "nostore" else 0
    e(f"s_waitcnt vmcnt({16 + n_all})")
    e("s_barrier")
    extra = body_head(e, epi, n_all)
    iteration(e, "first", diag, extra)
    e(f"s_sub_u32 s{S_LOOP}, s{S_KT}, 3")
    e("s_branch " + e.L("kloop"))
    # ---- no successor ----
    e.label(e.L("final"))
    iteration(e, "penult", diag, pre=pre_out)
    iteration(e, "last", diag)
    for _ in range(3):
        e("s_nop 7")
    if diag != "noepi":
        epilogue_store(e, epi)
    e.label(e.L("end"))
    e("s_waitcnt vmcnt(0)")
    e("s_endpgm")
    PLAIN_DIAG = None
    BFIRST = True
    SERPENTINE = False
    LOAD_POLICY = ("", "")
    SPLIT = True
    PLAIN_B2, PLAIN_DMA = B2_SLOT, DMA_SLOTS
    return e.text()


# deferred epilogue: stores issued at the tile boundary, then per successor K-step 0..3
N_IMMEDIATE = 6
DEFER_SPLIT = [7, 7, 6, 6]
DEFER_LONG = [2] * 13
V_STASH = V_EPI                 # 26 packed stores x 4 VGPRs = v[144:247]
V_ETMP = SET0_A                 # readout temps (the fragment sets are free until the successor's body_head)


def tile_boundary(e):
    for v in (V_RA0, V_RA1, V_RB0, V_RB1):       # fragment bases back at stage 0
        e(f"v_and_b32 v{v}, 0xffff, v{v}")
    for _ in range(3):                            # MFMA -> v_accvgpr_read wait states
        e("s_nop 7")


PLAIN_DIAG = None      # measurement builds of the plain kernel: "nostore" (pack, no stores), "nopack" (store, no pack)


def pack_row(e, epi, i, r, t, dst):
    """output row (i, r) of this wave: 8 accumulators -> (+ bias) -> 4 packed bf16 pairs in v[dst:dst+3]"""
    if PLAIN_DIAG == "nopack":
        return
    for j in range(8):
        e(f"v_accvgpr_read_b32 v{t + j}, a{(i * 8 + j) * 4 + r}")
    if epi == "bias":
        for j in range(8):
            e(f"v_add_f32 v{t + j}, v{t + j}, v{V_BIAS + j}")
    for p in range(4):
        e(f"v_cvt_pk_bf16_f32 v{dst + p}, v{t + 2 * p}, v{t + 2 * p + 1}")


STORE_POLICY = " nt"    # cache-policy modifier of the C stores: streaming (measured +1-2 % on wide N)


def store_row(i, r, src):
    if PLAIN_DIAG == "nostore":
        return []
    return [f"s_mul_i32 s{S_SOFFC}, s{S_LDC2}, {16 * i + r}",
            f"buffer_store_dwordx4 {vr(src)}, v{V_CO}, {sr(S_SRDC, 4)}, s{S_SOFFC} offen{STORE_POLICY}"]


def epilogue_stash(e, epi):
    """the first N_IMMEDIATE output rows stored now, the rest packed into V_STASH; returns their store groups"""
    assert N_IMMEDIATE + sum(DEFER_SPLIT) == 32 and V_STASH + 4 * sum(DEFER_SPLIT) <= V_BIAS
    groups = []
    for idx in range(32):
        i, r = divmod(idx, 4)
        t = V_ETMP + (idx % 4) * 12
        if idx < N_IMMEDIATE:
            pack_row(e, epi, i, r, t, t + 8)
            for ins in store_row(i, r, t + 8):
                e(ins)
        else:
            dst = V_STASH + 4 * (idx - N_IMMEDIATE)
            pack_row(e, epi, i, r, t, dst)
            groups.append(store_row(i, r, dst))
    return groups


def epilogue_store(e, epi):
    """all 32 output rows of this wave stored at once"""
    for idx in range(32):
        i, r = divmod(idx, 4)
        t = V_EPI + (idx % 4) * 12
        pack_row(e, epi, i, r, t, t + 8)
        for ins in store_row(i, r, t + 8):
            e(ins)


def set_srd(e, srd, ptr, row0, ld, nr):
    e(f"s_mul_i32 s{S_T0}, s{row0}, s{ld}")
    e(f"s_mul_hi_u32 s{S_T1}, s{row0}, s{ld}")
    e(f"s_lshl_b64 s[{S_T0}:{S_T1}], s[{S_T0}:{S_T1}], 1")
    e(f"s_add_u32 s{srd}, s{ptr}, s{S_T0}")
    e(f"s_addc_u32 s{srd + 1}, s{ptr + 1}, s{S_T1}")
    e(f"s_lshl_b32 s{nr}, s{ld}, 9")               # 256 rows * 2 bytes
    e(f"s_mov_b32 s{srd + 2}, s{nr}")
    e(f"s_mov_b32 s{srd + 3}, 0x20000")


KERNARG_SIZE = 112
LDS_BYTES = {}          # kernels that use LDS beyond the two operand stages


def metadata(name):
    args = []
    off = 0
    for _ in range(6):
        args.append(f"""      - .address_space:  global
        .offset:         {off}
        .size:           8
        .value_kind:     global_buffer""")
        off += 8
    for _ in range(16):
        args.append(f"""      - .offset:         {off}
        .size:           4
        .value_kind:     by_value""")
        off += 4
    return f"""  - .agpr_count:     256
    .args:
{chr(10).join(args)}
    .group_segment_fixed_size: {LDS_BYTES.get(name, 2 * STAGE)}
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
		.amdhsa_group_segment_fixed_size {LDS_BYTES.get(name, 2 * STAGE)}
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



# ----------------------------------------------------------------------------------------------------
# weight-gradient form (TN): dW partials.  C[s] (M x N fp32) = A[k, :]^T B[k, :] summed over the split's K
# rows, A (Ktot x M) and B (Ktot x N) TOKEN-major (the activations and output grads exactly as the forward
# and backward hold them: no transposed copies).  One workgroup per (tile, split) unit.
#
# The operand image of a K-step is [64 k-rows][256 columns] in the 8-row x 32-column subtile layout
# (cdna_hip_programming.md T10 (a)):  off(row, ch) = 2048 (row >> 3) + 512 (ch >> 2) + 64 (row & 7)
# + 16 ((ch & 3) ^ ((row >> 2) & 3))  per 128-column half (16 KB), so one LDS-DMA instruction (1 KB, lane-
# linear) fills 8 rows x 64 columns from whole 128-B lines, and an MFMA fragment (16 columns x 8 k) is two
# ds_read_b64_tr_b16 (rows 8g..8g+3 / +4..7 of the k-group g, delivered column-major = the operand layout),
# conflict-free.  The fragment's read address is base(rd, i & 1) + 512 (i >> 1) + 8192 h: 4 bases per
# operand.  Output: the standard 16x16 accumulator layout (lane holds column 16 j + c of rows 16 i + 4 g + r),
# stored as fp32 dwords into the split's partial slab; csrc/kernels/elementwise.hip splitk_accum folds the
# slabs into the fp32 weight grad (deterministic).
# ----------------------------------------------------------------------------------------------------
TN = False
TN_BFIRST = True     # B's transposed reads, image release and DMA ahead of A's: 0.6-1.2 % on the three large
                     # weight-grad shapes, 1.8 % slower on the small K163840 M1024 N1024 (profiles/r5_asm_wgrad_tn_bfirst)
V_TRA = 5            # A transposed-read bases (rd, i parity): v5..v8
V_TRB = 144          # B bases: v144..v147
V_TNT = 148          # TN temps v148..v159
S_STEPA, S_STEPB, S_SPLIT = 79, 80, 81
TN_SET1_SLOTS = list(range(16)) + [18 + 2 * n for n in range(16)]     # 16 A reads, then 16 B reads
TN_BA_SLOT, TN_BB_SLOT = 21, 52
TN_ONEBAR = False    # (measurement build tn_onebar: one stage-release barrier after all 32 reads, then the 16 DMAs)
TN_B2_SLOT = 50
TN_ONEBAR_DMA_SLOTS = [52 + round(4.8 * n) for n in range(16)]   # 52 .. 124
TN_DMA_SLOTS = [23 + 4 * n for n in range(8)] + [56 + round(9.7 * n) for n in range(8)]   # 23..51, 56..124


def tn_frag_reads(set_a, set_b, h):
    out = []
    for base, dst in ((V_TRA, set_a), (V_TRB, set_b)):
        for i in range(8):
            for rd in range(2):
                out.append(f"ds_read_b64_tr_b16 v[{dst + 4 * i + 2 * rd}:{dst + 4 * i + 2 * rd + 1}], "
                           f"v{base + 2 * rd + (i & 1)} offset:{8192 * h + 512 * (i >> 1)}")
    return out


def tn_lane_setup(e):
    T = V_TNT
    # ---- transposed-read bases: lane l = 16 g + 4 q + p:
    #      2048 g + 64 (q + 4 rd) + 16 ((2 ipar + (p >> 1)) ^ ((2 g + rd) & 3)) + 8 (p & 1) + 16 KB (wave half)
    # (v0 is the workgroup-wide thread id: every lane field is masked to the wave's 64)
    e(f"v_lshrrev_b32 v{T}, 4, v{V_TID}")
    e(f"v_and_b32 v{T}, 3, v{T}")                            # g
    e(f"v_lshrrev_b32 v{T + 1}, 2, v{V_TID}")
    e(f"v_and_b32 v{T + 1}, 3, v{T + 1}")                    # q
    e(f"v_lshrrev_b32 v{T + 2}, 1, v{V_TID}")
    e(f"v_and_b32 v{T + 2}, 1, v{T + 2}")                    # p >> 1
    e(f"v_and_b32 v{T + 3}, 1, v{V_TID}")                    # p & 1
    e(f"v_lshlrev_b32 v{T + 4}, 11, v{T}")                   # 2048 g
    e(f"v_lshl_add_u32 v{T + 4}, v{T + 1}, 6, v{T + 4}")      # + 64 q
    e(f"v_lshl_add_u32 v{T + 4}, v{T + 3}, 3, v{T + 4}")      # + 8 (p & 1)
    e(f"v_lshlrev_b32 v{T + 5}, 1, v{T}")                    # 2 g
    e(f"s_lshr_b32 s{S_T0}, s{S_WAVE}, 1")
    e(f"s_lshl_b32 s{S_T0}, s{S_T0}, 14")                    # A half: 16 KB wm
    e(f"s_and_b32 s{S_T1}, s{S_WAVE}, 1")
    e(f"s_lshl_b32 s{S_T1}, s{S_T1}, 14")
    e(f"s_add_u32 s{S_T1}, s{S_T1}, {B_IMG}")                # B half: B_IMG + 16 KB wn
    for rd in range(2):
        for ipar in range(2):
            k = 2 * rd + ipar
            e(f"v_add_u32 v{T + 6}, {rd}, v{T + 5}")
            e(f"v_and_b32 v{T + 6}, 3, v{T + 6}")            # (2 g + rd) & 3
            e(f"v_add_u32 v{T + 7}, {2 * ipar}, v{T + 2}")    # 2 ipar + (p >> 1)
            e(f"v_xor_b32 v{T + 6}, v{T + 6}, v{T + 7}")
            e(f"v_lshl_add_u32 v{T + 6}, v{T + 6}, 4, v{T + 4}")
            if rd:
                e(f"v_add_u32 v{T + 6}, 256, v{T + 6}")      # rows + 4: 64 * 4
            e(f"v_add_u32 v{V_TRA + k}, s{S_T0}, v{T + 6}")
            e(f"v_add_u32 v{V_TRB + k}, s{S_T1}, v{T + 6}")
    # ---- DMA sources: lane t -> row r = (t >> 2) & 7, subtile t >> 5, slot t & 3, b = (t >> 4) & 1:
    #      r ld2 + 64 (t >> 5) + 16 (slot ^ (2 Rpar + b)) + wave part 32 (q & 1) ld2 + 256 (q >> 1)
    e(f"v_lshrrev_b32 v{T}, 2, v{V_TID}")
    e(f"v_and_b32 v{T}, 7, v{T}")                            # r
    e(f"v_lshrrev_b32 v{T + 1}, 5, v{V_TID}")
    e(f"v_and_b32 v{T + 1}, 1, v{T + 1}")
    e(f"v_lshlrev_b32 v{T + 1}, 6, v{T + 1}")                # 64 sub
    e(f"v_and_b32 v{T + 2}, 3, v{V_TID}")                    # slot
    e(f"v_lshrrev_b32 v{T + 3}, 4, v{V_TID}")
    e(f"v_and_b32 v{T + 3}, 1, v{T + 3}")                    # b
    for par, (ga, gb) in enumerate(((V_GA0, V_GB0), (V_GA1, V_GB1))):
        e(f"v_add_u32 v{T + 4}, {2 * par}, v{T + 3}")
        e(f"v_xor_b32 v{T + 4}, v{T + 2}, v{T + 4}")
        e(f"v_lshl_add_u32 v{T + 4}, v{T + 4}, 4, v{T + 1}")  # 64 sub + 16 chunk
        e(f"v_mov_b32 v{ga}, v{T + 4}")
        e(f"v_mov_b32 v{gb}, v{T + 4}")
    for g_regs, ld, offs in (((V_GA0, V_GA1), S_LDA, S_OFFA), ((V_GB0, V_GB1), S_LDB, S_OFFB)):
        e(f"s_lshl_b32 s{S_T2}, s{ld}, 1")                   # ld2
        e(f"s_and_b32 s{S_T0}, s{S_WAVE}, 1")
        e(f"s_mul_i32 s{S_T0}, s{S_T0}, s{S_T2}")
        e(f"s_lshl_b32 s{S_T0}, s{S_T0}, 5")                 # 32 (q & 1) ld2
        e(f"s_lshr_b32 s{S_T1}, s{S_WAVE}, 1")
        e(f"s_lshl_b32 s{S_T1}, s{S_T1}, 8")
        e(f"s_add_u32 s{S_T0}, s{S_T0}, s{S_T1}")             # + 256 (q >> 1)
        for gr in g_regs:
            e(f"v_mad_u32_u24 v{gr}, v{T}, s{S_T2}, v{gr}")
            e(f"v_add_u32 v{gr}, s{S_T0}, v{gr}")
        for s_ in range(8):
            e(f"s_mul_i32 s{offs + s_}, s{S_T2}, {8 * (s_ >> 1)}")
            if s_ & 1:
                e(f"s_add_u32 s{offs + s_}, s{offs + s_}, 128")
    # ---- epilogue: (128 wm + 4 g) ldc4 + (128 wn + c) 4
    e(f"v_lshrrev_b32 v{T}, 4, v{V_TID}")
    e(f"v_and_b32 v{T}, 3, v{T}")
    e(f"v_lshlrev_b32 v{T}, 2, v{T}")                        # 4 g
    e(f"s_lshr_b32 s{S_T0}, s{S_WAVE}, 1")
    e(f"s_lshl_b32 s{S_T0}, s{S_T0}, 7")
    e(f"v_add_u32 v{T}, s{S_T0}, v{T}")
    e(f"v_mul_lo_u32 v{V_CO}, v{T}, s{S_LDC2}")              # S_LDC2 holds ldc * 4 in this kernel
    e(f"v_and_b32 v{T}, 15, v{V_TID}")
    e(f"s_and_b32 s{S_T1}, s{S_WAVE}, 1")
    e(f"s_lshl_b32 s{S_T1}, s{S_T1}, 7")
    e(f"v_add_u32 v{T}, s{S_T1}, v{T}")
    e(f"v_lshl_add_u32 v{V_CO}, v{T}, 2, v{V_CO}")


def div_const_free(e, q, r, n, d, mag):
    """s[q] = s[n] / s[d], s[r] = s[n] % s[d] with s[mag] = magic(s[d]) (0 when s[d] == 1)"""
    e(f"s_mul_hi_u32 s{q}, s{n}, s{mag}")
    e(f"s_cmp_eq_u32 s{mag}, 0")
    e(f"s_cselect_b32 s{q}, s{n}, s{q}")
    e(f"s_mul_i32 s{r}, s{q}, s{d}")
    e(f"s_sub_u32 s{r}, s{n}, s{r}")


def add64(e, srd, lo, hi):
    e(f"s_add_u32 s{srd}, s{srd}, s{lo}")
    e(f"s_addc_u32 s{srd + 1}, s{srd + 1}, s{hi}")


def mul64(e, a, b):
    """s[T0:T1] = s[a] * s[b] (64-bit)"""
    e(f"s_mul_i32 s{S_T0}, s{a}, s{b}")
    e(f"s_mul_hi_u32 s{S_T1}, s{a}, s{b}")


def kernel_tn(name, diag=None):
    global TN_BFIRST, TN_ONEBAR
    TN_BFIRST = diag != "tn_afirst"
    TN_ONEBAR = diag == "tn_onebar"
    try:
        return _kernel_tn(name, None if diag in ("tn_afirst", "tn_onebar") else diag)
    finally:
        TN_BFIRST, TN_ONEBAR = True, False


def _one_barrier(dg, gen):
    """measurement build "nosplit" of a fused kernel: one stage-release barrier (SPLIT off while it is generated)"""
    global SPLIT
    if dg != "nosplit":
        return gen(dg)
    SPLIT = False
    try:
        return gen(None)
    finally:
        SPLIT = True


def _kernel_tn(name, diag=None):
    global TN
    TN = True
    e = Emitter(name)
    e(f"s_load_dwordx8 {sr(S_A, 8)}, s[0:1], 0x0")          # A B C AUX0
    e(f"s_load_dwordx8 {sr(S_M, 8)}, s[0:1], 0x30")         # M N K lda ldb ldc tiles_n units
    e(f"s_load_dword s{S_GRID}, s[0:1], 0x50")
    e(f"v_lshrrev_b32 v{V_T}, 6, v{V_TID}")
    e("s_nop 1")
    e(f"v_readfirstlane_b32 s{S_WAVE}, v{V_T}")
    e("s_nop 1")
    e("s_waitcnt lgkmcnt(0)")
    e(f"s_lshr_b32 s{S_KT}, s{S_K}, 6")
    e(f"s_lshl_b32 s{S_LDC2}, s{S_LDC}, 2")                 # fp32 output: ldc * 4
    e(f"s_cmp_lt_u32 s{S_KT}, 4")
    e("s_cbranch_scc1 " + e.L("end"))
    e(f"s_bitcmp1_b32 s{S_KT}, 0")
    e("s_cbranch_scc1 " + e.L("end"))
    # ---- unit: XCD-major when the grid is a multiple of 8 (an XCD's CUs take consecutive units: the same
    #      split's neighbouring tiles, whose operand slices they share in L2) ----
    e(f"s_and_b32 s{S_T0}, s{S_GRID}, 7")
    e(f"s_mov_b32 s{S_TILE}, s{S_WG}")
    e(f"s_cmp_eq_u32 s{S_T0}, 0")
    e("s_cbranch_scc0 " + e.L("unit"))
    e(f"s_and_b32 s{S_T0}, s{S_WG}, 7")
    e(f"s_lshr_b32 s{S_T1}, s{S_GRID}, 3")
    e(f"s_mul_i32 s{S_T0}, s{S_T0}, s{S_T1}")
    e(f"s_lshr_b32 s{S_T1}, s{S_WG}, 3")
    e(f"s_add_u32 s{S_TILE}, s{S_T0}, s{S_T1}")
    e.label(e.L("unit"))
    e(f"s_cmp_lt_u32 s{S_TILE}, s{S_NT}")
    e("s_cbranch_scc0 " + e.L("end"))
    # tiles = (M / 256) tiles_n; split = unit / tiles, tile = unit % tiles; (tm, tni) = tile / tiles_n
    e(f"s_lshr_b32 s{S_T3}, s{S_M}, 8")
    e(f"s_mul_i32 s{S_G8}, s{S_T3}, s{S_TN}")                # tiles
    magic(e, S_MAGG, S_G8)
    e(f"s_cmp_lt_u32 s{S_G8}, 2")
    e(f"s_cselect_b32 s{S_MAGG}, 0, s{S_MAGG}")
    div_const_free(e, S_SPLIT, S_T2, S_TILE, S_G8, S_MAGG)
    e(f"s_mov_b32 s{S_ROWREM}, s{S_T2}")                    # tile
    magic(e, S_MAGR, S_TN)
    e(f"s_cmp_lt_u32 s{S_TN}, 2")
    e(f"s_cselect_b32 s{S_MAGR}, 0, s{S_MAGR}")
    div_const_free(e, S_TM, S_TNI, S_ROWREM, S_TN, S_MAGR)
    e(f"s_lshl_b32 s{S_ROW0}, s{S_TM}, 8")
    e(f"s_lshl_b32 s{S_COL0}, s{S_TNI}, 8")
    # ---- operand resources: base + split K rows + the tile's column block (no bounds: host-checked) ----
    e(f"s_mul_i32 s{S_T3}, s{S_SPLIT}, s{S_K}")             # first K row of the split
    for srd, ptr, ld, col, step in ((S_SRDA, S_A, S_LDA, S_ROW0, S_STEPA), (S_SRDB, S_B, S_LDB, S_COL0, S_STEPB)):
        e(f"s_mov_b32 s{srd}, s{ptr}")
        e(f"s_mov_b32 s{srd + 1}, s{ptr + 1}")
        mul64(e, S_T3, ld)
        e(f"s_lshl_b64 s[{S_T0}:{S_T1}], s[{S_T0}:{S_T1}], 1")
        add64(e, srd, S_T0, S_T1)
        e(f"s_lshl_b32 s{S_T0}, s{col}, 1")
        e(f"s_add_u32 s{srd}, s{srd}, s{S_T0}")
        e(f"s_addc_u32 s{srd + 1}, s{srd + 1}, 0")
        e(f"s_mov_b32 s{srd + 2}, -1")
        e(f"s_mov_b32 s{srd + 3}, 0x20000")
        e(f"s_lshl_b32 s{step}, s{ld}, 7")                  # 64 rows * 2 bytes
    # ---- partial slab: C + (split M N + row0 ldc + col0) * 4 ----
    e(f"s_mov_b32 s{S_SRDC}, s{S_C}")
    e(f"s_mov_b32 s{S_SRDC + 1}, s{S_C + 1}")
    e(f"s_mul_i32 s{S_T3}, s{S_M}, s{S_N}")
    mul64(e, S_SPLIT, S_T3)
    e(f"s_lshl_b64 s[{S_T0}:{S_T1}], s[{S_T0}:{S_T1}], 2")
    add64(e, S_SRDC, S_T0, S_T1)
    mul64(e, S_ROW0, S_LDC)
    e(f"s_add_u32 s{S_T0}, s{S_T0}, s{S_COL0}")
    e(f"s_addc_u32 s{S_T1}, s{S_T1}, 0")
    e(f"s_lshl_b64 s[{S_T0}:{S_T1}], s[{S_T0}:{S_T1}], 2")
    add64(e, S_SRDC, S_T0, S_T1)
    e(f"s_mov_b32 s{S_SRDC + 2}, -1")
    e(f"s_mov_b32 s{S_SRDC + 3}, 0x20000")
    e(f"s_lshl_b32 s{S_MBASE}, s{S_WAVE}, 13")
    tn_lane_setup(e)
    prologue_dma(e)
    e("s_waitcnt vmcnt(16)")
    e("s_barrier")
    for ins in frag_reads(SET0_A, SET0_B, 0):
        e(ins)
    e("s_waitcnt lgkmcnt(0)")
    iteration(e, "first", diag)
    e(f"s_sub_u32 s{S_LOOP}, s{S_KT}, 3")
    e.label(e.L("kloop"))
    iteration(e, "loop", diag)
    e(f"s_sub_u32 s{S_LOOP}, s{S_LOOP}, 1")
    e(f"s_cmp_eq_u32 s{S_LOOP}, 0")
    e("s_cbranch_scc0 " + e.L("kloop"))
    iteration(e, "penult", diag)
    iteration(e, "last", diag)
    for _ in range(3):
        e("s_nop 7")
    # ---- fp32 partial tile: lane holds column 16 j + c of rows 16 i + 4 g + r ----
    n = 0
    for i in range(8):
        for r in range(4):
            e(f"s_mul_i32 s{S_SOFFC}, s{S_LDC2}, {16 * i + r}")
            for j in range(8):
                t = V_TNT + (n % 8)
                n += 1
                e(f"v_accvgpr_read_b32 v{t}, a{(i * 8 + j) * 4 + r}")
                e(f"buffer_store_dword v{t}, v{V_CO}, {sr(S_SRDC, 4)}, s{S_SOFFC} offen offset:{64 * j}")
    e.label(e.L("end"))
    e("s_waitcnt vmcnt(0)")
    e("s_endpgm")
    TN = False
    return e.text()



# ----------------------------------------------------------------------------------------------------
# FF-in GEMM + GEGLU forward: a = x W1^T + b1 (M x 2F, [value | gate] column order) and u = value * gelu(gate)
# (M x F).  The B operand is W1 with its rows interleaved in 4-row blocks [value j..j+3 | gate j..j+3] (host:
# ff_in_perm), so each lane's 8 columns of a row are the values AND the gates of 4 consecutive j: the lane
# writes `a` back in the ORIGINAL column order as two 8-byte chunks (value j / gate F + j: 16 lanes = one whole
# 128-byte line each) and computes its 4 u from the same registers -- no exchange, no reload.  Both are deferred
# like the plain kernel's stores: the packed bf16 row-groups (the numbers the unfused geglu kernel would read)
# wait in v[144:247] while the successor tile's K-steps 0..13 (unrolled: needs kt >= 16, K >= 1024; the host
# checks) store them and spread the gelu VALU over their MFMA gaps.  The tile's bias is loaded during its last
# K-step, so v[248:255] serve as the gelu temps meanwhile.
# ----------------------------------------------------------------------------------------------------

# ----------------------------------------------------------------------------------------------------
# K generality of the fused kernels: their successor tile's K-steps 0..13 are unrolled (the deferred epilogue
# work rides in those steps' MFMA gaps), so a tile needs kt >= 16 K-steps (K >= 1024) and, as every kernel
# here, an even count (the successor's steps 0 / 1 land in stages 0 / 1).  Steps 14 .. kt - 3 then run in the
# ordinary K-loop and penult / last in the shared tail: K = 1024 (d_model 1024) and K = 2048 (the ~1.3B
# config's d_model) take the same code.
# ----------------------------------------------------------------------------------------------------
FUSED_UNROLL = 14


def kt_guard(e):
    """leave (no work) unless kt >= FUSED_UNROLL + 2 and even (the host rejects other shapes too)"""
    e(f"s_cmp_lt_u32 s{S_KT}, {FUSED_UNROLL + 2}")
    e("s_cbranch_scc1 " + e.L("end"))
    e(f"s_bitcmp1_b32 s{S_KT}, 0")
    e("s_cbranch_scc1 " + e.L("end"))


def successor_rest(e):
    """after the unrolled successor steps 0..13: kt - 16 plain loop steps (none at K = 1024), then the tail"""
    e(f"s_sub_u32 s{S_LOOP}, s{S_KT}, {FUSED_UNROLL + 2}")
    e(f"s_cmp_eq_u32 s{S_LOOP}, 0")
    e("s_cbranch_scc1 " + e.L("tail"))
    e("s_branch " + e.L("kloop"))

S_SRDU = 84          # u resource (4)
S_SOFFV, S_GP, S_MASK7, S_F2, S_LDU2, S_RSQ2 = 88, 89, 90, 91, 92, 93
S_AUX1, S_LDU = 22, 21
V_CU, V_COG = 13, 14                 # u store base, `a` gate-chunk base (value base: V_CO)
GE_T = V_BIAS                        # gelu temps v248..v254 (the packed u goes over the row-group's values)
GE_SPLIT = [2] * 12 + [1, 1]         # deferred row-groups' u per successor K-step 0..13 (26)
GE_CONSTS = {"c_rsqrt2": 0x3F3504F3, "a5": 0x3F87DC22, "a4": 0xBFBA00E3, "a3": 0x3FB5F0E3, "a2": 0xBE91A98E,
             "a1": 0x3E827906, "nhl2e": 0xBF38AA3B}


def fix_trans_hazards(seq):
    """gfx950: a VALU reading the result of a transcendental (v_rcp / v_exp) in the NEXT instruction needs one
    wait state -- insert s_nop 0 only where the consumer immediately follows"""
    out = []
    for i, ins in enumerate(seq):
        out.append(ins)
        if ins.startswith(("v_rcp_f32", "v_exp_f32")) and i + 1 < len(seq):
            dst = ins.split()[1].rstrip(",")
            nxt = seq[i + 1]
            if re.search(rf"\b{dst}\b", nxt.split(None, 1)[1] if " " in nxt else ""):
                out.append("s_nop 0")
    return out


GE_A = (0x3EB2303A, 0xBDC45CA1, 0x3F3F7377)    # A-S 7.1.25 a1, a2, a3 (erf(z) = 1 - (a1 t + a2 t^2 + a3 t^3) e^-z^2)
V_GEA3 = 255                         # a3 in a VGPR for v_fmaak during the successor's K-steps (the bias is back in 'last')
V_GEA3_B = 80                        # ... and at the tile boundary (fragment set 1 is free there)


def ge_u(src, temps, uout, va3=V_GEA3):
    """u for the lane's 4 j from the packed row-group v[src..src+3] = [v0v1, v2v3, g0g1, g2g3]:
    value * gelu(gate), erf by Abramowitz-Stegun 7.1.25 (|error| <= 2.5e-5, far below bf16 resolution), packed
    into uout[0], uout[1]; ``va3``: the VGPR holding a3"""
    g, v, t1, t2, t3, t4, ue = temps
    c = GE_CONSTS
    out = []
    for k in range(4):
        rv, rg_ = src + (k >> 1), src + 2 + (k >> 1)
        if k & 1:
            out += [f"v_and_b32 v{g}, 0xffff0000, v{rg_}", f"v_and_b32 v{v}, 0xffff0000, v{rv}"]
        else:
            out += [f"v_lshlrev_b32 v{g}, 16, v{rg_}", f"v_lshlrev_b32 v{v}, 16, v{rv}"]
        out += [f"v_fma_f32 v{t1}, |v{g}|, s{S_GP}, 1.0",                     # 1 + p |x| / sqrt2
                f"v_rcp_f32 v{t1}, v{t1}",                                   # t
                f"v_mul_f32 v{t3}, {c['nhl2e']:#x}, v{g}",
                f"v_fmaak_f32 v{t2}, v{t1}, v{va3}, {GE_A[1]:#x}",
                f"v_mul_f32 v{t3}, v{t3}, v{g}",                             # -x^2 / 2 * log2 e
                f"v_fmaak_f32 v{t2}, v{t2}, v{t1}, {GE_A[0]:#x}",
                f"v_exp_f32 v{t3}, v{t3}",                                   # exp(-x^2 / 2)
                f"v_mul_f32 v{t2}, v{t2}, v{t1}",                            # poly
                f"v_fma_f32 v{t4}, -v{t2}, v{t3}, 1.0",                      # |erf|
                f"v_bfi_b32 v{t4}, s{S_MASK7}, v{t4}, v{g}",                 # copysign(., x)
                f"v_fma_f32 v{t4}, 0.5, v{t4}, 0.5",                         # cdf
                f"v_mul_f32 v{t4}, v{g}, v{t4}",                             # gelu
                f"v_mul_f32 v{t4}, v{v}, v{t4}"]                             # u
        if k & 1:
            out.append(f"v_cvt_pk_bf16_f32 v{uout[k >> 1]}, v{ue}, v{t4}")
        else:
            out.append(f"v_mov_b32 v{ue}, v{t4}")
    return fix_trans_hazards(out)


def ge_stores_a(i, r, src):
    """the row-group's value chunk (v[src:src+1]) and gate chunk (v[src+2:src+3]) of `a`"""
    return [f"s_mul_i32 s{S_SOFFC}, s{S_LDC2}, {16 * i + r}",
            f"buffer_store_dwordx2 v[{src}:{src + 1}], v{V_CO}, {sr(S_SRDC, 4)}, s{S_SOFFC} offen",
            f"buffer_store_dwordx2 v[{src + 2}:{src + 3}], v{V_COG}, {sr(S_SRDC, 4)}, s{S_SOFFC} offen"]


def geglu_lane_setup(e, diag=None):
    """per-lane bases of the geglu epilogue: `a` value / gate chunks in the original column order, u"""
    T0, T1 = V_T, V_T + 1
    # rows 128 wm + 4 g; value j = 64 wn + 4 c  (c = lane & 15)
    e(f"v_lshrrev_b32 v{T0}, 4, v{V_TID}")
    e(f"v_and_b32 v{T0}, 3, v{T0}")
    e(f"v_lshlrev_b32 v{T0}, 2, v{T0}")
    e(f"s_lshr_b32 s{S_T0}, s{S_WAVE}, 1")
    e(f"s_lshl_b32 s{S_T0}, s{S_T0}, 7")
    e(f"v_add_u32 v{T0}, s{S_T0}, v{T0}")                # row
    e(f"v_and_b32 v{T1}, 15, v{V_TID}")
    e(f"v_lshlrev_b32 v{T1}, 3, v{T1}")                  # 4 c columns * 2 bytes
    e(f"s_and_b32 s{S_T1}, s{S_WAVE}, 1")
    e(f"s_lshl_b32 s{S_T1}, s{S_T1}, 7")                # 64 wn * 2 bytes
    e(f"v_add_u32 v{T1}, s{S_T1}, v{T1}")
    e(f"v_mul_lo_u32 v{V_CO}, v{T0}, s{S_LDC2}")
    e(f"v_add_u32 v{V_CO}, v{V_CO}, v{T1}")
    if diag == "adjacent":      # measurement: gate chunk stored right after the value chunk (wrong layout)
        e(f"v_lshlrev_b32 v{T1}, 1, v{T1}")
        e(f"v_mul_lo_u32 v{V_CO}, v{T0}, s{S_LDC2}")
        e(f"v_add_u32 v{V_CO}, v{V_CO}, v{T1}")
        e(f"v_add_u32 v{V_COG}, 8, v{V_CO}")
    else:
        e(f"v_add_u32 v{V_COG}, s{S_F2}, v{V_CO}")
    e(f"v_mul_lo_u32 v{V_CU}, v{T0}, s{S_LDU2}")
    e(f"v_add_u32 v{V_CU}, v{V_CU}, v{T1}")


def setup_output_geglu():
    """(in penult's MFMA gaps) `a` resource of the finishing tile (S_ROW0, S_COL0): a + row0 ldc2 + col0 (its
    F-columns start at col0 / 2), u resource u + row0 ldu2 + col0, bias resource aux0 + col0 * 4"""
    out = []
    for srd, ptr, ld2 in ((S_SRDC, S_C, S_LDC2), (S_SRDU, S_AUX1, S_LDU2)):
        out += [f"s_mul_i32 s{S_T0}, s{S_ROW0}, s{ld2}", f"s_mul_hi_u32 s{S_T1}, s{S_ROW0}, s{ld2}",
                f"s_add_u32 s{S_T0}, s{S_T0}, s{S_COL0}", f"s_addc_u32 s{S_T1}, s{S_T1}, 0",
                f"s_add_u32 s{srd}, s{ptr}, s{S_T0}", f"s_addc_u32 s{srd + 1}, s{ptr + 1}, s{S_T1}",
                f"s_lshl_b32 s{srd + 2}, s{ld2}, 8", f"s_mov_b32 s{srd + 3}, 0x20000"]
    out += [f"s_lshl_b32 s{S_T0}, s{S_COL0}, 2", f"s_add_u32 s{S_SRDX}, s{S_AUX0}, s{S_T0}",
            f"s_addc_u32 s{S_SRDX + 1}, s{S_AUX0 + 1}, 0", f"s_mov_b32 s{S_SRDX + 2}, 1024",
            f"s_mov_b32 s{S_SRDX + 3}, 0x20000"]
    return out


BIAS_LOADS = [f"buffer_load_dwordx4 {vr(V_BIAS)}, v{V_BOFF}, {sr(S_SRDX, 4)}, 0 offen",
              f"buffer_load_dwordx4 {vr(V_BIAS + 4)}, v{V_BOFF}, {sr(S_SRDX, 4)}, 0 offen offset:16"]


def kernel_geglu(name, diag=None):
    global STORE_POLICY
    STORE_POLICY = ""
    e = Emitter(name)
    e(f"s_load_dwordx8 {sr(S_A, 8)}, s[0:1], 0x0")
    e(f"s_load_dwordx2 {sr(S_AUX1, 2)}, s[0:1], 0x20")
    e(f"s_load_dwordx8 {sr(S_M, 8)}, s[0:1], 0x30")
    e(f"s_load_dword s{S_GRID}, s[0:1], 0x50")
    e(f"s_load_dword s{S_LDU}, s[0:1], 0x54")
    e(f"v_lshrrev_b32 v{V_T}, 6, v{V_TID}")
    e("s_nop 1")
    e(f"v_readfirstlane_b32 s{S_WAVE}, v{V_T}")
    e("s_nop 1")
    e("s_waitcnt lgkmcnt(0)")
    e(f"s_lshr_b32 s{S_KT}, s{S_K}, 6")
    e(f"s_lshl_b32 s{S_LDC2}, s{S_LDC}, 1")
    e(f"s_lshl_b32 s{S_LDU2}, s{S_LDU}, 1")
    e(f"s_lshl_b32 s{S_F2}, s{S_LDU}, 1")               # 2 F bytes: the gate half of an `a` row (ld_aux = F)
    e(f"s_mov_b32 s{S_GP}, 0x3eaa540e")                  # 0.47047 / sqrt 2
    e(f"s_mov_b32 s{S_MASK7}, 0x7fffffff")
    kt_guard(e)
    lane_setup(e, "bias")
    geglu_lane_setup(e, diag)
    e(f"s_and_b32 s{S_T0}, s{S_WG}, 7")
    e(f"s_lshr_b32 s{S_T1}, s{S_GRID}, 3")
    e(f"s_mul_i32 s{S_T0}, s{S_T0}, s{S_T1}")
    e(f"s_lshr_b32 s{S_T1}, s{S_WG}, 3")
    e(f"s_add_u32 s{S_TILE}, s{S_T0}, s{S_T1}")
    e(f"s_cmp_lt_u32 s{S_TILE}, s{S_NT}")
    e("s_cbranch_scc0 " + e.L("end"))
    tile_order_setup(e)
    stagger_setup(e)
    emit_all(e, tile_coords())
    setup_operands(e)
    prologue_dma(e)
    e("s_waitcnt vmcnt(16)")
    e("s_barrier")
    body_head(e, "plain", 0)
    iteration(e, "first", None, 0)
    e(f"s_sub_u32 s{S_LOOP}, s{S_KT}, 3")
    e.label(e.L("kloop"))
    iteration(e, "loop")
    e(f"s_sub_u32 s{S_LOOP}, s{S_LOOP}, 1")
    e(f"s_cmp_eq_u32 s{S_LOOP}, 0")
    e("s_cbranch_scc0 " + e.L("kloop"))
    e.label(e.L("tail"))
    pre_out = setup_output_geglu()
    sub = Emitter(e.prefix)
    setup_operands(sub)
    pre_next = pre_out + next_tile() + [l.strip() for l in sub.lines]
    e(f"s_add_u32 s{S_T0}, s{S_TILE}, s{S_GRID}")
    e(f"s_cmp_lt_u32 s{S_T0}, s{S_NT}")
    e("s_cbranch_scc0 " + e.L("final"))
    iteration(e, "penult", None, prefetch=True, pre=pre_next)
    vm = iteration(e, "last", None, prefetch=True, work=BIAS_LOADS, work_span=(1, 4))
    after_bias = len(vm) - 1 - max(i for i, ins in enumerate(vm) if ins in BIAS_LOADS)
    e(f"s_waitcnt vmcnt({after_bias})")                  # this tile's bias is in
    tile_boundary(e)
    e(f"v_mov_b32 v{V_GEA3_B}, {GE_A[2]:#x}")
    # ---- boundary: pack every row-group (+ bias); the first N_IMMEDIATE stored and their u computed now ----
    stash = []
    n_imm_vmem = 0
    for idx in range(32):
        i, r = divmod(idx, 4)
        t = V_ETMP + (idx % 4) * 12
        if idx < N_IMMEDIATE:
            pack_row(e, "bias", i, r, t, t + 8)
            seq = ge_stores_a(i, r, t + 8)
            if diag not in ("nowork", "adjacent"):
                seq += ge_u(t + 8, (t, t + 1, t + 2, t + 3, t + 4, t + 5, t + 6), (t + 8, t + 9), V_GEA3_B)
                seq += [f"s_mul_i32 s{S_SOFFV}, s{S_LDU2}, {16 * i + r}",
                        f"buffer_store_dwordx2 v[{t + 8}:{t + 9}], v{V_CU}, {sr(S_SRDU, 4)}, s{S_SOFFV} offen"]
            emit_all(e, seq)
            n_imm_vmem += sum(1 for x in seq if x.startswith("buffer_"))
        else:
            dst = V_STASH + 4 * (idx - N_IMMEDIATE)
            pack_row(e, "bias", i, r, t, dst)
            stash.append((i, r, dst))
    e(f"v_mov_b32 v{V_GEA3}, {GE_A[2]:#x}")             # (over the bias: packed)
    e(f"s_waitcnt vmcnt({16 + n_imm_vmem})")             # the successor's step 0 landed
    e("s_barrier")
    body_head(e, "plain", 0)
    # ---- successor K-steps 0 .. 13, unrolled: `a` stores of the stashed row-groups and their u (gelu VALU +
    #      store), two row-groups per step ----
    ui = 0
    per_step_a = [2] * 13               # with each row-group's u, in the same step (over [7, 7, 6, 6]: see r5_asm_geglu_v4)
    ai = 0
    for t in range(FUSED_UNROLL):
        work = []
        if t < len(per_step_a):
            for (i, r, src) in stash[ai:ai + per_step_a[t]]:
                work += ge_stores_a(i, r, src)
            ai += per_step_a[t]
        if diag not in ("nowork", "adjacent"):
            for (i, r, src) in stash[ui:ui + GE_SPLIT[t]]:
                # (its `a` chunks were stored in this or an earlier step: the values may be overwritten)
                work += ge_u(src, tuple(GE_T + q for q in range(7)), (src, src + 1))
                work += [f"s_mul_i32 s{S_SOFFV}, s{S_LDU2}, {16 * i + r}",
                         f"buffer_store_dwordx2 v[{src}:{src + 1}], v{V_CU}, {sr(S_SRDU, 4)}, s{S_SOFFV} offen"]
            ui += GE_SPLIT[t]
        iteration(e, "first" if t == 0 else "loop", None, n_imm_vmem if t == 0 else 0, work=work,
                  work_span=(1, 118))
    successor_rest(e)
    e.label(e.L("final"))
    iteration(e, "penult", None, pre=pre_out)
    vm = iteration(e, "last", None, work=BIAS_LOADS, work_span=(1, 4))
    e("s_waitcnt vmcnt(0)")
    for _ in range(3):
        e("s_nop 7")
    e(f"v_mov_b32 v{V_GEA3_B}, {GE_A[2]:#x}")
    for idx in range(32):
        i, r = divmod(idx, 4)
        t = V_EPI + (idx % 4) * 12
        pack_row(e, "bias", i, r, t, t + 8)
        seq = ge_stores_a(i, r, t + 8)
        if diag not in ("nowork", "adjacent"):
            seq += ge_u(t + 8, (t, t + 1, t + 2, t + 3, t + 4, t + 5, t + 6), (t + 8, t + 9), V_GEA3_B)
            seq += [f"s_mul_i32 s{S_SOFFV}, s{S_LDU2}, {16 * i + r}",
                    f"buffer_store_dwordx2 v[{t + 8}:{t + 9}], v{V_CU}, {sr(S_SRDU, 4)}, s{S_SOFFV} offen"]
        emit_all(e, seq)
    e.label(e.L("end"))
    e("s_waitcnt vmcnt(0)")
    e("s_endpgm")
    STORE_POLICY = " nt"
    return e.text()



# ----------------------------------------------------------------------------------------------------
# QKV projection + 3-axis rotary written straight into the attention storage (q pre-scaled): qkv = h Wqkv^T
# (M x 3 H 64), each 64-column head block rotated pairwise by the (cos, sin) of its sequence position and stored
# as row st(p) of head (part, b, h) of the (3, B H, Np, 64) storage -- st(p) = p for text, Tp + the image
# position (transposed for the axial-column pattern, variant _col) otherwise.  A tile is 256 positions of ONE
# sample (host: n % 256 == 0) and 4 heads of one part.  The rotation runs on the stored bf16 values, as the
# unfused path (GEMM, then rope_fwd) does, so it is deferred like the plain stores: 8 row-groups rotated and
# stored at the tile boundary with (cos, sin) prefetched during the last K-step, 24 packed in v[144:239] and
# rotated / stored under the successor's K-steps 0..11 (their (cos, sin) loaded early in the same step).
# cs3 = (3, n + 1, 32, 2) fp32 (cos, sin) per rotary pair of q (scaled by 1/8), k and v (all three rotated).
# ----------------------------------------------------------------------------------------------------
S_SRDQ, S_SRDCS = 84, 88
S_QN, S_QT, S_QTP, S_QNP, S_QH, S_QLOGS, S_QP0, S_QMAGN = 92, 93, 94, 95, 96, 97, 98, 99
S_QBT, S_QHD = 82, 83
V_QLC, V_QPL, V_QCS = 13, 14, 15
QX = (9, 10, 11, 12)                 # rotation temps
Q_IMM = 8                            # row-groups rotated at the boundary
Q_BANKS = (240, 248)                 # (cos, sin) of the two row-groups of a successor step
Q_IMM_BANK = 176                     # the boundary row-groups' (cos, sin), prefetched in the last K-step


def qkv_setup_tile():
    """(penult's MFMA gaps) the finishing tile's sample b, first position p0, part / first head, and the
    storage and (cos, sin) resources"""
    T0, T1, T2, T3 = S_T0, S_T1, S_T2, S_T3
    return [f"s_mul_hi_u32 s{T0}, s{S_ROW0}, s{S_QMAGN}",          # b
            f"s_mul_i32 s{T1}, s{T0}, s{S_QN}",
            f"s_sub_u32 s{S_QP0}, s{S_ROW0}, s{T1}",                # p0
            f"s_cmp_ge_u32 s{S_COL0}, s{S_QHD}",
            f"s_cselect_b32 s{T1}, 1, 0",
            f"s_lshl_b32 s{T2}, s{S_QHD}, 1",
            f"s_cmp_ge_u32 s{S_COL0}, s{T2}",
            f"s_cselect_b32 s{T2}, 1, 0",
            f"s_add_u32 s{T1}, s{T1}, s{T2}",                       # part
            f"s_mul_i32 s{T2}, s{T1}, s{S_QHD}",
            f"s_sub_u32 s{T2}, s{S_COL0}, s{T2}",
            f"s_lshr_b32 s{T2}, s{T2}, 6",                          # first head of the tile
            f"s_mul_i32 s{T3}, s{T1}, s{S_QBT}",
            f"s_add_u32 s{T3}, s{T3}, s{T0}",
            f"s_mul_i32 s{T3}, s{T3}, s{S_QH}",
            f"s_add_u32 s{T3}, s{T3}, s{T2}",                       # global head index
            f"s_add_u32 s{T0}, s{S_QN}, 1",
            f"s_mul_i32 s{T0}, s{T0}, s{T1}",
            f"s_lshl_b32 s{T0}, s{T0}, 8",                          # part (n + 1) 256
            f"s_add_u32 s{S_SRDCS}, s{S_AUX0}, s{T0}",
            f"s_addc_u32 s{S_SRDCS + 1}, s{S_AUX0 + 1}, 0",
            f"s_mov_b32 s{S_SRDCS + 2}, -1",
            f"s_mov_b32 s{S_SRDCS + 3}, 0x20000",
            f"s_mul_i32 s{T2}, s{T3}, s{S_QNP}",
            f"s_mov_b32 s{T3}, 0",
            f"s_lshl_b64 s[{T2}:{T3}], s[{T2}:{T3}], 7",            # head * Np * 128 bytes
            f"s_add_u32 s{S_SRDQ}, s{S_C}, s{T2}",
            f"s_addc_u32 s{S_SRDQ + 1}, s{S_C + 1}, s{T3}",
            f"s_mov_b32 s{S_SRDQ + 2}, -1",
            f"s_mov_b32 s{S_SRDQ + 3}, 0x20000"]


def qkv_load(i, r, bank, tag):
    """(cos, sin) of the row-group's 4 pairs: v[bank:bank+7] (the byte offset goes through v[bank+4])"""
    return [f"v_add_u32 v{bank + 4}, s{S_QP0}, v{V_QPL}",
            f"v_add_u32 v{bank + 4}, {16 * i + r}, v{bank + 4}",          # position p
            f"v_lshl_add_u32 v{bank + 4}, v{bank + 4}, 8, v{V_QCS}",
            f"buffer_load_dwordx4 v[{bank}:{bank + 3}], v{bank + 4}, {sr(S_SRDCS, 4)}, 0 offen ; @{tag}",
            f"buffer_load_dwordx4 v[{bank + 4}:{bank + 7}], v{bank + 4}, {sr(S_SRDCS, 4)}, 0 offen offset:16 ; @{tag}"]


def qkv_rotate_store(i, r, src, bank, col):
    """rotate the packed row-group v[src:src+3] by v[bank:bank+7], then store it at its storage row"""
    x0, x1, ta, tb = QX
    out = []
    for k in range(4):
        cs_, sn = bank + 2 * k, bank + 2 * k + 1
        out += [f"v_lshlrev_b32 v{x0}, 16, v{src + k}",
                f"v_and_b32 v{x1}, 0xffff0000, v{src + k}",
                f"v_mul_f32 v{ta}, v{x1}, v{sn}",
                f"v_fma_f32 v{ta}, v{x0}, v{cs_}, -v{ta}",                  # x0 c - x1 s
                f"v_mul_f32 v{tb}, v{x0}, v{sn}",
                f"v_fma_f32 v{tb}, v{x1}, v{cs_}, v{tb}",                   # x1 c + x0 s
                f"v_cvt_pk_bf16_f32 v{src + k}, v{ta}, v{tb}"]
    p, st, t = bank, bank + 1, bank + 2
    out += [f"v_add_u32 v{p}, s{S_QP0}, v{V_QPL}",
            f"v_add_u32 v{p}, {16 * i + r}, v{p}",
            f"v_subrev_u32 v{st}, s{S_QT}, v{p}"]                           # image position k = p - T
    if col:
        out += [f"v_bfe_u32 v{t}, v{st}, 0, s{S_QLOGS}",
                f"v_lshlrev_b32 v{t}, s{S_QLOGS}, v{t}",
                f"v_lshrrev_b32 v{st}, s{S_QLOGS}, v{st}",
                f"v_add3_u32 v{st}, v{t}, v{st}, s{S_QTP}"]                 # Tp + (k % S) S + k / S
    else:
        out += [f"v_add_u32 v{st}, s{S_QTP}, v{st}"]                        # Tp + k
    out += [f"v_cmp_gt_u32 vcc, s{S_QT}, v{p}",
            f"v_cndmask_b32 v{st}, v{st}, v{p}, vcc",                       # text: row p
            f"v_lshl_add_u32 v{st}, v{st}, 7, v{V_QLC}",
            f"buffer_store_dwordx4 {vr(src)}, v{st}, {sr(S_SRDQ, 4)}, 0 offen"]
    return out


def qkv_lane_setup(e):
    T0, T1 = V_T, V_T + 1
    # V_QLC = (2 wn + (c >> 3)) Np 128 + 16 (c & 7);  V_QPL = 128 wm + 4 g;  V_QCS = 32 (c & 7)
    e(f"v_and_b32 v{T0}, 15, v{V_TID}")
    e(f"v_lshrrev_b32 v{T0}, 3, v{T0}")                  # c >> 3
    e(f"s_and_b32 s{S_T0}, s{S_WAVE}, 1")
    e(f"s_lshl_b32 s{S_T0}, s{S_T0}, 1")
    e(f"v_add_u32 v{T0}, s{S_T0}, v{T0}")                # head within the tile
    e(f"s_lshl_b32 s{S_T1}, s{S_QNP}, 7")
    e(f"v_mul_lo_u32 v{V_QLC}, v{T0}, s{S_T1}")
    e(f"v_and_b32 v{T1}, 7, v{V_TID}")
    e(f"v_lshlrev_b32 v{V_QCS}, 5, v{T1}")
    e(f"v_lshl_add_u32 v{V_QLC}, v{T1}, 4, v{V_QLC}")
    e(f"v_lshrrev_b32 v{T0}, 4, v{V_TID}")
    e(f"v_and_b32 v{T0}, 3, v{T0}")
    e(f"v_lshlrev_b32 v{T0}, 2, v{T0}")
    e(f"s_lshr_b32 s{S_T0}, s{S_WAVE}, 1")
    e(f"s_lshl_b32 s{S_T0}, s{S_T0}, 7")
    e(f"v_add_u32 v{V_QPL}, s{S_T0}, v{T0}")


def kernel_qkv(name, col):
    e = Emitter(name)
    e(f"s_load_dwordx8 {sr(S_A, 8)}, s[0:1], 0x0")
    e(f"s_load_dwordx8 {sr(S_M, 8)}, s[0:1], 0x30")
    e(f"s_load_dword s{S_GRID}, s[0:1], 0x50")
    e(f"s_load_dwordx2 s[{S_QN}:{S_QT}], s[0:1], 0x54")     # n, T
    e(f"s_load_dwordx2 s[{S_QTP}:{S_QNP}], s[0:1], 0x5c")   # Tp, Np
    e(f"s_load_dwordx2 s[{S_QH}:{S_QLOGS}], s[0:1], 0x64")  # H, log2 S
    e(f"v_lshrrev_b32 v{V_T}, 6, v{V_TID}")
    e("s_nop 1")
    e(f"v_readfirstlane_b32 s{S_WAVE}, v{V_T}")
    e("s_nop 1")
    e("s_waitcnt lgkmcnt(0)")
    e(f"s_lshr_b32 s{S_KT}, s{S_K}, 6")
    kt_guard(e)
    e(f"s_lshl_b32 s{S_QHD}, s{S_QH}, 6")                # H * 64 columns per part
    magic(e, S_QMAGN, S_QN)
    e(f"s_mul_hi_u32 s{S_QBT}, s{S_M}, s{S_QMAGN}")      # batch = M / n
    lane_setup(e, "plain")
    qkv_lane_setup(e)
    e(f"s_and_b32 s{S_T0}, s{S_WG}, 7")
    e(f"s_lshr_b32 s{S_T1}, s{S_GRID}, 3")
    e(f"s_mul_i32 s{S_T0}, s{S_T0}, s{S_T1}")
    e(f"s_lshr_b32 s{S_T1}, s{S_WG}, 3")
    e(f"s_add_u32 s{S_TILE}, s{S_T0}, s{S_T1}")
    e(f"s_cmp_lt_u32 s{S_TILE}, s{S_NT}")
    e("s_cbranch_scc0 " + e.L("end"))
    tile_order_setup(e)
    stagger_setup(e)
    emit_all(e, tile_coords())
    setup_operands(e)
    prologue_dma(e)
    e("s_waitcnt vmcnt(16)")
    e("s_barrier")
    body_head(e, "plain", 0)
    iteration(e, "first", None, 0)
    e(f"s_sub_u32 s{S_LOOP}, s{S_KT}, 3")
    e.label(e.L("kloop"))
    iteration(e, "loop")
    e(f"s_sub_u32 s{S_LOOP}, s{S_LOOP}, 1")
    e(f"s_cmp_eq_u32 s{S_LOOP}, 0")
    e("s_cbranch_scc0 " + e.L("kloop"))
    e.label(e.L("tail"))
    pre_out = qkv_setup_tile()
    sub = Emitter(e.prefix)
    setup_operands(sub)
    pre_next = pre_out + next_tile() + [l.strip() for l in sub.lines]
    imm_loads = []
    for idx in range(Q_IMM):
        i, r = divmod(idx, 4)
        imm_loads += qkv_load(i, r, Q_IMM_BANK + 8 * idx, "imm")

    def boundary(final):
        vm = iteration(e, "last", None, prefetch=not final, work=imm_loads, work_span=(1, 17))
        last_ld = max(k for k, ins in enumerate(vm) if ins.endswith("; @imm"))
        e(f"s_waitcnt vmcnt({len(vm) - 1 - last_ld})")
        if not final:
            tile_boundary(e)
        else:
            for _ in range(3):
                e("s_nop 7")
        n_vm = 0
        for idx in range(Q_IMM):
            i, r = divmod(idx, 4)
            t = V_ETMP + (idx % 4) * 12
            pack_row(e, "plain", i, r, t, t + 8)
            seq = qkv_rotate_store(i, r, t + 8, Q_IMM_BANK + 8 * idx, col)
            emit_all(e, seq)
            n_vm += 1
        return n_vm

    e(f"s_add_u32 s{S_T0}, s{S_TILE}, s{S_GRID}")
    e(f"s_cmp_lt_u32 s{S_T0}, s{S_NT}")
    e("s_cbranch_scc0 " + e.L("final"))
    iteration(e, "penult", None, prefetch=True, pre=pre_next)
    n_vm = boundary(False)
    stash = []
    for idx in range(Q_IMM, 32):
        i, r = divmod(idx, 4)
        dst = V_STASH + 4 * (idx - Q_IMM)
        pack_row(e, "plain", i, r, V_ETMP, dst)
        stash.append((i, r, dst))
    e(f"s_waitcnt vmcnt({16 + n_vm})")                   # the successor's step 0 landed
    e("s_barrier")
    body_head(e, "plain", 0)
    for t in range(FUSED_UNROLL):
        loads, comp = [], []
        for b_, (i, r, src) in enumerate(stash[2 * t:2 * t + 2] if t < 12 else []):
            tag = f"q{b_}"
            loads += qkv_load(i, r, Q_BANKS[b_], tag)
            comp += [f"@vmwait:{tag}"] + qkv_rotate_store(i, r, src, Q_BANKS[b_], col)
        iteration(e, "first" if t == 0 else "loop", None, n_vm if t == 0 else 0, work=loads, work_span=(1, 4),
                  work2=comp, work2_span=(60, 118))
    successor_rest(e)
    e.label(e.L("final"))
    iteration(e, "penult", None, pre=pre_out)
    boundary(True)
    for idx in range(Q_IMM, 32):
        i, r = divmod(idx, 4)
        t = V_EPI + (idx % 4) * 12
        pack_row(e, "plain", i, r, t, t + 8)
        emit_all(e, qkv_load(i, r, Q_BANKS[0], "f") + ["s_waitcnt vmcnt(0)"] +
                 qkv_rotate_store(i, r, t + 8, Q_BANKS[0], col))
    e.label(e.L("end"))
    e("s_waitcnt vmcnt(0)")
    e("s_endpgm")
    return e.text()


# ----------------------------------------------------------------------------------------------------
# FF-out dgrad + GEGLU backward: du = dy W2 (M x F; A = dy (M x K), B = W2^T (F x K), K = d_model), then with the
# FF-in pre-activation a (M x 2F, [value | gate], aux0):  da_value = du gelu(gate), da_gate = du value gelu'(gate)
# into dh (M x 2F, C; ldc = 2F, ld_aux = F), and the FF-in bias gradient's column sums per 128-row block into
# part (M / 128 x 2F fp32, aux1; the host folds it).  du is rounded to bf16 first, as the unfused path stores
# it.  Each lane's row-group (8 consecutive du columns of one row) needs the same 8 columns of a's value and
# gate halves: two 16-byte loads, two 16-byte stores, no exchange.  The GEGLU backward is VALU-heavy (~27
# instructions per element), so it runs under the successor tile's MFMAs: 7 row-groups at the tile boundary,
# 17 with du packed in v[144:211] and 8 with du in the LDS above the two operand stages (32 KB), processed two
# per successor K-step 0..13 (unrolled: K >= 1024) with their `a` chunks loaded one K-step ahead (two banks of
# 16 VGPRs).  Column sums: each element's (da, dg) pair is folded over lanes g, g + 2 by v_permlane32_swap into
# 8 running sums; at the tile's end v_permlane16_swap folds g, g + 1 and each lane stores 4 of the 128-row
# block's sums (16 bytes).
# ----------------------------------------------------------------------------------------------------
GB_STASH, GB_LDS = 20, 8
GB_IMM = 32 - GB_STASH - GB_LDS                 # 4 row-groups processed at the tile boundary
V_GBANK = 224                                   # a chunks of the two row-groups in flight (A, B): 2 x 8 VGPRs
V_GSUM = 240                                    # 8 fp32 column sums
V_GDA = 248                                     # da0 da1 dg0 dg1
V_GA3 = 252                                     # the polynomial's leading coefficient (fmaak needs it in a VGPR)
GX2 = (80, 81, 82, 83)                          # second chain's temps at the tile boundary (fragment set 1)
V_GCOG, V_GPO, V_GLDS = 13, 14, 0               # gate chunk offset, part offset, LDS stash base (over v0)
GX = (10, 11, 12, 15)                           # temps
S_SRDAA, S_SRDP = S_SRDX, 84                    # a / part resources of the finishing tile
S_GSOF = (88, 89)
S_GMASK, S_GPR, S_GNH, S_GC2, S_GF = 90, 91, 92, 93, 94
LDS_GB = 2 * STAGE
for _n in ("dalle_gemm_nt_geglu_bwd", "dalle_gemm_diag_gbwd_novalu", "dalle_gemm_diag_gbwd_nomem",
           "dalle_gemm_diag_gbwd_nosplit"):
    LDS_BYTES[_n] = LDS_GB + 256 * 16 * GB_LDS       # 160 KB: the whole LDS


def fix_valu_hazards(seq):
    """fix_trans_hazards, plus gfx950's two wait states between a VALU write and a v_permlane*_swap reading
    (and rewriting) that VGPR"""
    seq = fix_trans_hazards(seq)
    out = []
    for ins in seq:
        if ins.startswith("v_permlane"):
            regs = [x.strip() for x in ins.split(None, 1)[1].split(",")]
            waits = 0
            for prev in reversed(out):
                if prev.startswith("s_nop"):
                    waits += int(prev.split()[1]) + 1
                    continue
                if prev.startswith("v_") and prev.split(None, 1)[1].split(",")[0].strip() in regs:
                    if waits < 2:
                        out.append(f"s_nop {1 - waits}")
                    break
                waits += 1
                if waits >= 2:
                    break
        out.append(ins)
    return out


GB_A = (0x3F5F5377, 0xBE761A62, 0x3FEFF2C3)    # A-S 7.1.25 a1, a2, a3, each times sqrt(2 pi)
GB_DIAG = None          # measurement builds: "novalu" (no GELU math), "nomem" (no `a` loads / dh stores)


def gb_load(idx, bank, sof, tag):
    """the row-group's value / gate chunks of `a` into v[bank:bank+7]"""
    i, r = divmod(idx, 4)
    if GB_DIAG == "nomem":
        return [f"s_mul_i32 s{sof}, s{S_LDC2}, {16 * i + r}"]
    return [f"s_mul_i32 s{sof}, s{S_LDC2}, {16 * i + r}",
            f"buffer_load_dwordx4 {vr(bank)}, v{V_CO}, {sr(S_SRDAA, 4)}, s{sof} offen nt ; @{tag}",
            f"buffer_load_dwordx4 {vr(bank + 4)}, v{V_GCOG}, {sr(S_SRDAA, 4)}, s{sof} offen nt ; @{tag}"]


def gb_compute(idx, du, bank, sof, temps2=None):
    """da / dg of the row-group (du packed bf16 in v[du:du+3], a's value / gate chunks in v[bank:bank+7]) into
    v[bank:bank+7], stored; the pair-folded values added to the column sums.  ``temps2``: four more temps --
    the two columns of each pair then run as two interleaved dependency chains (the tile boundary, where no
    MFMA gaps hide the chain latency)"""
    out = []
    unpack = lambda dst, src, h: (f"v_and_b32 v{dst}, 0xffff0000, v{src}" if h else f"v_lshlrev_b32 v{dst}, 16, v{src}")

    def chain(k2, h, temps):
        x, x1, x2, x3 = temps
        da, dg = V_GDA + h, V_GDA + 2 + h
        if GB_DIAG == "novalu":
            return [unpack(x3, du + k2, h), unpack(x, bank + k2, h), f"v_mul_f32 v{da}, v{x3}, v{x}",
                    unpack(x1, bank + 4 + k2, h), f"v_mul_f32 v{dg}, v{x3}, v{x1}"]
        # erf(|x| / sqrt2) by Abramowitz-Stegun 7.1.25 (|error| <= 2.5e-5, far below bf16 resolution) with
        # its coefficients scaled by sqrt(2 pi), so the exponential it multiplies is the normal pdf itself
        return [unpack(x, bank + 4 + k2, h),                                   # gate
                f"v_fma_f32 v{x1}, |v{x}|, s{S_GPR}, 1.0",                      # 1 + p |x| / sqrt2
                f"v_rcp_f32 v{x1}, v{x1}",                                       # t
                f"v_mul_f32 v{x3}, s{S_GNH}, v{x}",
                f"v_fma_f32 v{x3}, v{x3}, v{x}, s{S_GC2}",                      # log2 pdf
                f"v_fmaak_f32 v{x2}, v{x1}, v{V_GA3}, {GB_A[1]:#x}",
                f"v_exp_f32 v{x3}, v{x3}",                                       # pdf
                f"v_fmaak_f32 v{x2}, v{x2}, v{x1}, {GB_A[0]:#x}",
                f"v_mul_f32 v{x2}, v{x2}, v{x1}",                                # poly sqrt(2 pi)
                f"v_fma_f32 v{x1}, -v{x2}, v{x3}, 1.0",                          # |erf|
                f"v_bfi_b32 v{x1}, s{S_GMASK}, v{x1}, v{x}",                      # copysign(., x)
                f"v_fma_f32 v{x1}, 0.5, v{x1}, 0.5",                              # cdf
                f"v_fma_f32 v{x2}, v{x}, v{x3}, v{x1}",                           # gelu' = cdf + x pdf
                f"v_mul_f32 v{x1}, v{x}, v{x1}",                                  # gelu
                unpack(x3, du + k2, h),                                           # du
                f"v_mul_f32 v{da}, v{x3}, v{x1}",
                unpack(x, bank + k2, h),                                          # value
                f"v_mul_f32 v{x2}, v{x2}, v{x}",
                f"v_mul_f32 v{dg}, v{x3}, v{x2}"]

    for k2 in range(4):
        c0, c1 = chain(k2, 0, GX), chain(k2, 1, temps2 or GX)
        if temps2:
            out += [ins for pair in zip(c0, c1) for ins in pair]
        else:
            out += c0 + c1
        out += [f"v_cvt_pk_bf16_f32 v{bank + k2}, v{V_GDA}, v{V_GDA + 1}",
                f"v_cvt_pk_bf16_f32 v{bank + 4 + k2}, v{V_GDA + 2}, v{V_GDA + 3}"]
        for h in range(2):
            da, dg, sm = V_GDA + h, V_GDA + 2 + h, V_GSUM + 2 * k2 + h
            out += [f"v_permlane32_swap_b32 v{da}, v{dg}",                        # lanes < 32: da (g, g + 2)
                    f"v_add_f32 v{sm}, v{sm}, v{da}",                             # lanes >= 32: dg
                    f"v_add_f32 v{sm}, v{sm}, v{dg}"]
    i, r = divmod(idx, 4)
    out += [f"s_mul_i32 s{sof}, s{S_LDC2}, {16 * i + r}"]
    if GB_DIAG != "nomem":
        out += [f"buffer_store_dwordx4 {vr(bank)}, v{V_CO}, {sr(S_SRDC, 4)}, s{sof} offen nt",
                f"buffer_store_dwordx4 {vr(bank + 4)}, v{V_GCOG}, {sr(S_SRDC, 4)}, s{sof} offen nt"]
    return fix_valu_hazards(out)


def gb_finish():
    """fold the sums over lanes g, g + 1 and store this lane's 4 of them; zero the sums for the next tile"""
    out = ["s_nop 1"]
    for k in range(4):
        out += [f"v_permlane16_swap_b32 v{V_GSUM + k}, v{V_GSUM + 4 + k}",
                f"v_add_f32 v{V_GSUM + k}, v{V_GSUM + k}, v{V_GSUM + 4 + k}"]
    out.append(f"buffer_store_dwordx4 {vr(V_GSUM)}, v{V_GPO}, {sr(S_SRDP, 4)}, 0 offen")
    out += [f"v_mov_b32 v{V_GSUM + 4 + k}, 0" for k in range(4)] + [f"v_mov_b32 v{V_GSUM + k}, 0" for k in range(4)]
    return fix_valu_hazards(out)


def gb_lane_setup(e):
    """gate chunk offset, part offset, LDS stash base; zero sums.  The sums' lanes after both folds:
    (lane >> 5) selects value / gate columns, (lane >> 4) & 1 the upper 4 of the lane's 8 columns."""
    T0, T1 = V_T, V_T + 1
    e(f"s_lshl_b32 s{S_T0}, s{S_GF}, 1")
    e(f"v_add_u32 v{V_GCOG}, s{S_T0}, v{V_CO}")              # + F columns * 2 bytes
    # part: wm ldc 4 + (lane >> 5) F 4 + (128 wn + 8 c + 4 ((lane >> 4) & 1)) 4
    e(f"v_and_b32 v{T0}, 15, v{V_TID}")
    e(f"v_lshlrev_b32 v{V_GPO}, 5, v{T0}")                    # 8 c * 4
    e(f"v_lshrrev_b32 v{T0}, 4, v{V_TID}")
    e(f"v_and_b32 v{T0}, 1, v{T0}")
    e(f"v_lshl_add_u32 v{V_GPO}, v{T0}, 4, v{V_GPO}")
    e(f"v_lshrrev_b32 v{T0}, 5, v{V_TID}")
    e(f"v_and_b32 v{T0}, 1, v{T0}")
    e(f"s_lshl_b32 s{S_T0}, s{S_GF}, 2")
    e(f"v_mul_lo_u32 v{T0}, v{T0}, s{S_T0}")
    e(f"v_add_u32 v{V_GPO}, v{V_GPO}, v{T0}")
    e(f"s_and_b32 s{S_T0}, s{S_WAVE}, 1")
    e(f"s_lshl_b32 s{S_T0}, s{S_T0}, 9")                     # 128 wn * 4
    e(f"v_add_u32 v{V_GPO}, s{S_T0}, v{V_GPO}")
    e(f"s_lshr_b32 s{S_T0}, s{S_WAVE}, 1")
    e(f"s_mul_i32 s{S_T0}, s{S_T0}, s{S_LDC}")
    e(f"s_lshl_b32 s{S_T0}, s{S_T0}, 2")                     # wm ldc * 4
    e(f"v_add_u32 v{V_GPO}, s{S_T0}, v{V_GPO}")
    e(f"v_lshlrev_b32 v{V_GLDS}, 4, v{V_TID}")
    e(f"v_add_u32 v{V_GLDS}, {LDS_GB}, v{V_GLDS}")           # + 16 tid (v0 is not needed past here)
    for k in range(8):
        e(f"v_mov_b32 v{V_GSUM + k}, 0")
    e(f"v_mov_b32 v{V_GA3}, {GB_A[2]:#x}")


def gb_setup_tile():
    """(penult's MFMA gaps) dh, a and part resources of the finishing tile"""
    out = []
    for srd, ptr in ((S_SRDC, S_C), (S_SRDAA, S_AUX0)):
        out += [f"s_mul_i32 s{S_T0}, s{S_ROW0}, s{S_LDC}", f"s_mul_hi_u32 s{S_T1}, s{S_ROW0}, s{S_LDC}",
                f"s_add_u32 s{S_T0}, s{S_T0}, s{S_COL0}", f"s_addc_u32 s{S_T1}, s{S_T1}, 0",
                f"s_lshl_b64 s[{S_T0}:{S_T1}], s[{S_T0}:{S_T1}], 1",
                f"s_add_u32 s{srd}, s{ptr}, s{S_T0}", f"s_addc_u32 s{srd + 1}, s{ptr + 1}, s{S_T1}",
                f"s_lshl_b32 s{srd + 2}, s{S_LDC2}, 8", f"s_mov_b32 s{srd + 3}, 0x20000"]
    out += [f"s_lshr_b32 s{S_T0}, s{S_ROW0}, 7", f"s_mul_i32 s{S_T0}, s{S_T0}, s{S_LDC}",
            f"s_add_u32 s{S_T0}, s{S_T0}, s{S_COL0}", f"s_mov_b32 s{S_T1}, 0",
            f"s_lshl_b64 s[{S_T0}:{S_T1}], s[{S_T0}:{S_T1}], 2",
            f"s_add_u32 s{S_SRDP}, s{S_AUX1}, s{S_T0}", f"s_addc_u32 s{S_SRDP + 1}, s{S_AUX1 + 1}, s{S_T1}",
            f"s_lshl_b32 s{S_SRDP + 2}, s{S_LDC}, 3", f"s_mov_b32 s{S_SRDP + 3}, 0x20000"]
    return out


def gb_plan():
    """deferred row-groups per successor K-step: (idx, du location) with location ('v', reg) or ('l', k)"""
    deferred = [(GB_IMM + s, ("v", V_STASH + 4 * s)) for s in range(GB_STASH)] + \
               [(GB_IMM + GB_STASH + k, ("l", k)) for k in range(GB_LDS)]
    per = [2] * 14
    assert sum(per) == len(deferred)
    plan, k = [], 0
    for n in per:
        plan.append(deferred[k:k + n])
        k += n
    return plan


def kernel_geglu_bwd(name, diag=None):
    global GB_DIAG
    GB_DIAG = diag
    e = Emitter(name)
    e(f"s_load_dwordx8 {sr(S_A, 8)}, s[0:1], 0x0")
    e(f"s_load_dwordx2 {sr(S_AUX1, 2)}, s[0:1], 0x20")
    e(f"s_load_dwordx8 {sr(S_M, 8)}, s[0:1], 0x30")
    e(f"s_load_dword s{S_GRID}, s[0:1], 0x50")
    e(f"s_load_dword s{S_GF}, s[0:1], 0x54")
    e(f"v_lshrrev_b32 v{V_T}, 6, v{V_TID}")
    e("s_nop 1")
    e(f"v_readfirstlane_b32 s{S_WAVE}, v{V_T}")
    e("s_nop 1")
    e("s_waitcnt lgkmcnt(0)")
    e(f"s_lshr_b32 s{S_KT}, s{S_K}, 6")
    e(f"s_lshl_b32 s{S_LDC2}, s{S_LDC}, 1")
    e(f"s_mov_b32 s{S_GMASK}, 0x7fffffff")
    e(f"s_mov_b32 s{S_GPR}, 0x3eaa540e")                 # 0.47047 / sqrt 2
    e(f"s_mov_b32 s{S_GNH}, {GE_CONSTS['nhl2e']:#x}")     # -log2(e) / 2
    e(f"s_mov_b32 s{S_GC2}, 0xbfa9b21d")                 # log2(1 / sqrt(2 pi))
    kt_guard(e)
    lane_setup(e, "plain")
    gb_lane_setup(e)
    e(f"s_and_b32 s{S_T0}, s{S_WG}, 7")
    e(f"s_lshr_b32 s{S_T1}, s{S_GRID}, 3")
    e(f"s_mul_i32 s{S_T0}, s{S_T0}, s{S_T1}")
    e(f"s_lshr_b32 s{S_T1}, s{S_WG}, 3")
    e(f"s_add_u32 s{S_TILE}, s{S_T0}, s{S_T1}")
    e(f"s_cmp_lt_u32 s{S_TILE}, s{S_NT}")
    e("s_cbranch_scc0 " + e.L("end"))
    tile_order_setup(e)
    stagger_setup(e)
    emit_all(e, tile_coords())
    setup_operands(e)
    prologue_dma(e)
    e("s_waitcnt vmcnt(16)")
    e("s_barrier")
    body_head(e, "plain", 0)
    iteration(e, "first", None, 0)
    e(f"s_sub_u32 s{S_LOOP}, s{S_KT}, 3")
    e.label(e.L("kloop"))
    iteration(e, "loop")
    e(f"s_sub_u32 s{S_LOOP}, s{S_LOOP}, 1")
    e(f"s_cmp_eq_u32 s{S_LOOP}, 0")
    e("s_cbranch_scc0 " + e.L("kloop"))
    e.label(e.L("tail"))
    pre_out = gb_setup_tile()
    sub = Emitter(e.prefix)
    setup_operands(sub)
    pre_next = pre_out + next_tile() + [l.strip() for l in sub.lines]
    imm_loads = []
    for idx in range(GB_IMM):
        imm_loads += gb_load(idx, V_STASH + 8 * idx, S_GSOF[idx % 2], "imm")
    plan = gb_plan()
    banks = (V_GBANK, V_GBANK + 8)

    def load(t, b, tag):
        return gb_load(plan[t][b][0], banks[b], S_GSOF[b], tag)

    def compute(t, b):
        idx, loc = plan[t][b]
        du = loc[1] if loc[0] == "v" else V_STASH + 4 * loc[1]
        return gb_compute(idx, du, banks[b], S_GSOF[b])

    def after_last(vm, tag):
        tagged = [k for k, ins in enumerate(vm) if ins.endswith("; @" + tag)]
        return len(vm) - 1 - max(tagged) if tagged else 0     # (none in the nomem measurement build)

    def boundary_imm(vm_pen, vm_last):
        e(f"s_waitcnt vmcnt({after_last(vm_pen, 'imm') + len(vm_last)})")   # the immediate row-groups' a chunks
        n = 0
        for idx in range(GB_IMM):
            i, r = divmod(idx, 4)
            t = V_ETMP + (idx % 4) * 12
            pack_row(e, "plain", i, r, t, t + 8)
            emit_all(e, gb_compute(idx, t + 8, V_STASH + 8 * idx, S_GSOF[idx % 2], temps2=GX2))
            n += 2
        return n

    e(f"s_add_u32 s{S_T0}, s{S_TILE}, s{S_GRID}")
    e(f"s_cmp_lt_u32 s{S_T0}, s{S_NT}")
    e("s_cbranch_scc0 " + e.L("final"))
    # ---- successor: 4 row-groups now, 28 under its K-steps 0..13: in step t, row-group A's `a` chunks were
    #      loaded in step t - 1 (after its A was stored), B's at the start of step t ----
    vm_pen = iteration(e, "penult", None, prefetch=True, pre=pre_next, work=imm_loads, work_span=(20, 60))
    vm_last = iteration(e, "last", None, prefetch=True, work=load(0, 0, "a0"), work_span=(1, 8))
    tile_boundary(e)
    n_st = boundary_imm(vm_pen, vm_last)
    for idx in range(GB_IMM, 32):
        i, r = divmod(idx, 4)
        t = V_ETMP + (idx % 4) * 12
        if idx < GB_IMM + GB_STASH:
            pack_row(e, "plain", i, r, t, V_STASH + 4 * (idx - GB_IMM))
        else:
            pack_row(e, "plain", i, r, t, t + 8)
            e(f"ds_write_b128 v{V_GLDS}, {vr(t + 8)} offset:{4096 * (idx - GB_IMM - GB_STASH)}")
    e(f"s_waitcnt vmcnt({len(vm_last) + n_st})")         # the successor's step 0 landed
    e("s_barrier")
    body_head(e, "plain", 0)
    prev_wait = after_last(vm_last, "a0") + n_st
    for t in range(FUSED_UNROLL):
        at = []
        if t + 1 < 14:
            lds_next = [(idx, loc) for idx, loc in plan[t + 1] if loc[0] == "l"]
            for n, (idx, loc) in enumerate(lds_next):
                # into the du registers of an already processed VGPR-stashed row-group
                at.append((47 + n, f"ds_read_b128 {vr(V_STASH + 4 * loc[1])}, v{V_GLDS} offset:{4096 * loc[1]}"))
            if lds_next:
                at.append((62, "s_waitcnt lgkmcnt(0)"))
        comp_a = [f"@vmwait_prev:{prev_wait}"] + compute(t, 0)
        next_a = load(t + 1, 0, f"a{t + 1}") if t + 1 < 14 else []
        comp_b = [f"@vmwait:b{t}"] + compute(t, 1) + (gb_finish() if t == 13 else [])
        vm = iteration(e, "first" if t == 0 else "loop", None, n_st if t == 0 else 0, work=load(t, 1, f"b{t}"),
                       work_span=(1, 4), work2=comp_a, work2_span=(8, 62), at=at,
                       more=((next_a, (63, 65)), (comp_b, (66, 120))))
        if next_a:
            prev_wait = after_last(vm, f"a{t + 1}")
    successor_rest(e)
    # ---- no successor: 4 row-groups, then the other 28 in three load batches ----
    e.label(e.L("final"))
    vm_pen = iteration(e, "penult", None, pre=pre_out, work=imm_loads, work_span=(20, 60))
    vm_last = iteration(e, "last", None)
    for _ in range(3):
        e("s_nop 7")
    boundary_imm(vm_pen, vm_last)
    rest = list(range(GB_IMM, 32))
    for batch in (rest[:10], rest[10:19], rest[19:]):
        for n, idx in enumerate(batch):
            emit_all(e, gb_load(idx, V_STASH + 8 * n, S_GSOF[n % 2], "f"))
        e("s_waitcnt vmcnt(0)")
        for n, idx in enumerate(batch):
            i, r = divmod(idx, 4)
            t = V_ETMP + (n % 4) * 12
            pack_row(e, "plain", i, r, t, t + 8)
            emit_all(e, gb_compute(idx, t + 8, V_STASH + 8 * n, S_GSOF[n % 2], temps2=GX2))
    emit_all(e, gb_finish())
    e.label(e.L("end"))
    e("s_waitcnt vmcnt(0)")
    e("s_endpgm")
    GB_DIAG = None
    return e.text()


KERNELS = [("dalle_gemm_nt_plain", "plain", None), ("dalle_gemm_nt_bias", "bias", None), ("dalle_gemm_tn_wgrad", "tn", None),
           ("dalle_gemm_nt_geglu", "geglu", None), ("dalle_gemm_nt_qkv_row", "qkv", 0), ("dalle_gemm_nt_qkv_col", "qkv", 1),
           ("dalle_gemm_nt_geglu_bwd", "geglu_bwd", None)]
DIAG_KERNELS = [(f"dalle_gemm_diag_{d}", "plain", d) for d in ("noepi", "nodma", "split", "nostagger", "nostore",
                                                                  "nopack", "defer4", "afirst", "serp", "ant", "abnt", "l2store", "b2_33",
                                                                  "dma_dense")] + [
    ("dalle_gemm_diag_geglu_nowork", "geglu", "nowork"), ("dalle_gemm_diag_geglu_adjacent", "geglu", "adjacent"),
    ("dalle_gemm_diag_gbwd_novalu", "geglu_bwd", "novalu"), ("dalle_gemm_diag_gbwd_nomem", "geglu_bwd", "nomem"),
    ("dalle_gemm_diag_tn_nodma", "tn", "nodma"), ("dalle_gemm_diag_tn_afirst", "tn", "tn_afirst"),
    ("dalle_gemm_diag_tn_onebar", "tn", "tn_onebar"), ("dalle_gemm_diag_geglu_nosplit", "geglu", "nosplit"),
    ("dalle_gemm_diag_gbwd_nosplit", "geglu_bwd", "nosplit")]


# The schedule knobs the kernel builders read are module globals (the measurement variants flip them for one
# build).  Every kernel is generated from a fresh copy of their defaults, so a kernel's code depends only on
# (name, epilogue, variant) -- never on which kernels were generated before it (tests/test_asm_cpu.py
# generates the production set in two opposite orders, diagnostic variants interleaved, and compares).
_KNOBS = ("SERPENTINE", "LOAD_POLICY", "BFIRST", "STAGGER", "SPLIT", "STORE_POLICY", "PLAIN_DIAG", "PLAIN_B2",
          "PLAIN_DMA", "TN", "TN_BFIRST", "TN_ONEBAR", "GB_DIAG")


def _knob_defaults():
    g = globals()
    g.setdefault("PLAIN_B2", B2_SLOT)
    g.setdefault("PLAIN_DMA", DMA_SLOTS)
    return {k: (list(g[k]) if isinstance(g[k], list) else g[k]) for k in _KNOBS}


def generate(name, epi, dg=None):
    """the assembly of one kernel, from the default knobs (restored afterwards as well)"""
    g = globals()
    saved = _knob_defaults()
    g.update({k: (list(v) if isinstance(v, list) else v) for k, v in _DEFAULT_KNOBS.items()})
    try:
        if epi == "tn":
            return kernel_tn(name, dg)
        if epi == "geglu":
            return _one_barrier(dg, lambda d: kernel_geglu(name, d))
        if epi == "qkv":
            return kernel_qkv(name, dg)
        if epi == "geglu_bwd":
            return _one_barrier(dg, lambda d: kernel_geglu_bwd(name, d))
        return kernel(name, epi, dg)
    finally:
        g.update(_DEFAULT_KNOBS if saved is None else saved)


def main(out, diag=False, kernels=None):
    """``kernels``: (name, epilogue, variant) list to emit (default: the production set, + the diagnostic
    variants when ``diag``)"""
    parts = ['\t.amdgcn_target "amdgcn-amd-amdhsa--gfx950"', "\t.amdhsa_code_object_version 6", "\t.text"]
    metas = []
    for name, epi, dg in (kernels if kernels is not None else (KERNELS + DIAG_KERNELS if diag else KERNELS)):
        parts += [f"\t.globl\t{name}", "\t.p2align\t8", f"\t.type\t{name},@function", f"{name}:"]
        parts.append(generate(name, epi, dg))
        parts.append(f"\t.size\t{name}, .-{name}")
        parts.append(descriptor(name))
        metas.append(metadata(name))
    parts.append("\t.amdgpu_metadata\n---\namdhsa.kernels:\n" + "".join(metas)
                 + "amdhsa.target:   amdgcn-amd-amdhsa--gfx950\namdhsa.version:\n  - 1\n  - 2\n...\n\n\t.end_amdgpu_metadata")
    with open(out, "w") as f:
        f.write("\n".join(parts) + "\n")


_DEFAULT_KNOBS = _knob_defaults()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else "gemm_gfx950.s",
         diag="--diag" in sys.argv)
