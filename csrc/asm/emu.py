#!/usr/bin/env python3
"""Functional emulator of the generated gfx950 GEMM kernels (csrc/asm/gen_gemm.py) on the CPU.

Runs one workgroup (4 waves) instruction by instruction -- SALU, the VALU subset the generator emits,
LDS reads (ds_read_b128, ds_read_b64_tr_b16), LDS-DMA buffer loads, buffer stores, v_mfma_f32_16x16x32_bf16 --
against numpy "global memory" whose every access is bounds-checked against the tensors that were passed
in: a kernel that would fault on the GPU raises here with the instruction and the address instead.  Waves run
in turn between barriers (a barrier is a rendezvous of all 4); memory operations complete at issue, so
s_waitcnt is a no-op (the emulator checks addressing and data layout, not the timing of the schedule).

    python csrc/asm/emu.py            # self-test: the NT and TN kernels on small shapes vs numpy
"""
import os
import re
import struct
import sys

import numpy as np

M32 = 0xFFFFFFFF


def bf16_to_f32(u16):
    return (u16.astype(np.uint32) << 16).view(np.float32)


def f32_to_bf16(f):
    u = np.asarray(f, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    return r


class Memory:
    """global memory: named byte buffers at fake base addresses; every access is range-checked"""

    def __init__(self):
        self.bufs = []   # (base, bytearray-like np.uint8 array, name)
        self.next = 0x1000_0000

    def alloc(self, arr, name):
        b = np.frombuffer(np.ascontiguousarray(arr).tobytes(), dtype=np.uint8).copy()
        base = self.next
        self.next += (len(b) + 0xFFFFF) & ~0xFFFFF
        self.next += 0x100000
        self.bufs.append((base, b, name))
        return base

    def find(self, addr, n):
        for base, b, name in self.bufs:
            if base <= addr and addr + n <= base + len(b):
                return b, addr - base
        raise RuntimeError(f"out-of-bounds global access at {addr:#x} (+{n})")

    def read(self, addr, n):
        b, o = self.find(addr, n)
        return b[o:o + n]

    def write(self, addr, data):
        b, o = self.find(addr, len(data))
        b[o:o + len(data)] = data

    def get(self, base, dtype, shape):
        for bb, b, name in self.bufs:
            if bb == base:
                return b.view(dtype).reshape(shape)
        raise KeyError(base)


def parse_kernel(asm_text, name):
    lines = asm_text.split("\n")
    start = lines.index(f"{name}:") + 1
    code, labels = [], {}
    for l in lines[start:]:
        if l.startswith("\t.size"):
            break
        s = l.strip()
        if not s or s.startswith(";"):
            continue
        if s.endswith(":"):
            labels[s[:-1]] = len(code)
            continue
        code.append(s)
    return code, labels


def reg_range(tok):
    """'v[16:19]' -> (16, 4); 'v5' -> (5, 1); 's[24:27]' -> (24, 4); 'a[0:3]' -> (0, 4)"""
    m = re.match(r"^[vsa]\[(\d+):(\d+)\]$", tok)
    if m:
        return int(m.group(1)), int(m.group(2)) - int(m.group(1)) + 1
    return int(tok[1:]), 1


class Wave:
    def __init__(self, wid):
        self.v = np.zeros((256, 64), dtype=np.uint32)
        self.a = np.zeros((256, 64), dtype=np.float32)
        self.s = np.zeros(108, dtype=np.uint64)
        self.m0 = 0
        self.scc = 0
        self.vcc = np.zeros(64, dtype=bool)
        self.pc = 0
        self.done = False
        self.v[0] = np.arange(64) + 64 * wid


class Workgroup:
    def __init__(self, code, labels, mem, kernarg, wg_id, lds_bytes=160 * 1024, lds_alloc=131072):
        self.code, self.labels, self.mem = code, labels, mem
        self.lds = np.zeros(lds_bytes, dtype=np.uint8)
        self.lds_alloc = lds_alloc
        self.waves = [Wave(w) for w in range(4)]
        ka = mem.alloc(np.frombuffer(kernarg, dtype=np.uint8), "kernarg")
        for w in self.waves:
            w.s[0] = ka & M32
            w.s[1] = ka >> 32
            w.s[2] = wg_id

    # ---- operand helpers ----
    def sval(self, w, tok):
        tok = tok.strip()
        if tok == "m0":
            return w.m0
        if tok.startswith("s") and tok[1:].isdigit():
            return int(w.s[int(tok[1:])]) & M32
        if tok.startswith("0x"):
            return int(tok, 16) & M32
        return int(tok) & M32

    def vval(self, w, tok):
        """per-lane uint32 operand: VGPR, SGPR (broadcast) or constant (integer, or an inline float like 0.5)"""
        tok = tok.strip()
        if tok.startswith("v") and tok[1:].isdigit():
            return w.v[int(tok[1:])].astype(np.uint64)
        if re.match(r"^-?\d+\.\d+$", tok):
            return np.full(64, int(np.float32(float(tok)).view(np.uint32)), dtype=np.uint64)
        return np.full(64, self.sval(w, tok), dtype=np.uint64)

    def fval(self, w, tok):
        """per-lane fp32 operand with an optional neg (-v) or abs (|v|) modifier"""
        tok = tok.strip()
        if tok.startswith("|") and tok.endswith("|"):
            return np.abs(self.vval(w, tok[1:-1]).astype(np.uint32).view(np.float32))
        neg = tok.startswith("-v")
        r = self.vval(w, tok[1:] if neg else tok).astype(np.uint32).view(np.float32)
        return -r if neg else r

    def run_wave(self, w):
        """run until a barrier or the end; returns 'barrier' or 'end'"""
        code = self.code
        while True:
            if w.pc >= len(code):
                w.done = True
                return "end"
            ins = code[w.pc]
            w.pc += 1
            r = self.step(w, ins)
            if r:
                return r

    def run(self, max_rounds=10 ** 7):
        for _ in range(max_rounds):
            states = [self.run_wave(w) if not w.done else "end" for w in self.waves]
            if all(s == "end" for s in states):
                return
            if any(s == "end" for s in states) and any(s == "barrier" for s in states):
                raise RuntimeError("barrier mismatch: some waves ended while others wait")
        raise RuntimeError("too many barrier rounds")

    def step(self, w, ins):
        op, _, rest = ins.partition(" ")
        # split args but keep modifiers (offen, lds, offset:N, nt) separately
        toks = [t.strip() for t in rest.split(",")] if rest else []
        mods = []
        if toks:
            last = toks[-1].split()
            toks[-1] = last[0]
            mods = last[1:]
        d = lambda i=0: int(toks[i][1:])
        S = w.s
        if op == "s_endpgm":
            w.done = True
            return "end"
        if op == "s_barrier":
            return "barrier"
        if op in ("s_nop", "s_waitcnt"):
            return None
        if op in ("s_load_dwordx8", "s_load_dwordx2", "s_load_dword"):
            base, n = reg_range(toks[0])
            addr = (int(S[int(toks[1][2:].split(":")[0])]) | (int(S[int(toks[1][2:].split(":")[0]) + 1]) << 32)) + int(toks[2], 16)
            data = self.mem.read(addr, 4 * n).view(np.uint32)
            for i in range(n):
                S[base + i] = int(data[i])
            return None
        if op.startswith("s_"):
            return self.salu(w, op, toks)
        if op.startswith("v_mfma"):
            return self.mfma(w, toks)
        if op.startswith("v_"):
            return self.valu(w, op, toks)
        if op.startswith("ds_read"):
            return self.ds_read(w, op, toks, mods)
        if op == "ds_write_b128":
            off = 0
            for m in mods:
                if m.startswith("offset:"):
                    off = int(m[7:])
            src = reg_range(toks[1])[0]
            addr = w.v[int(toks[0][1:])].astype(np.int64) + off
            for l in range(64):
                a = int(addr[l])
                assert a % 16 == 0 and a + 16 <= self.lds_alloc, f"ds_write_b128 address {a}"
                self.lds[a:a + 16] = w.v[src:src + 4, l].astype(np.uint32).view(np.uint8)
            return None
        if op.startswith("buffer_"):
            return self.buffer(w, op, toks, mods)
        raise RuntimeError("unsupported: " + ins)

    def salu(self, w, op, t):
        S = w.s
        val = lambda x: self.sval(w, x)

        def setd(v):
            if t[0] == "m0":
                w.m0 = v & M32
            else:
                S[int(t[0][1:])] = v & M32
        if op == "s_mov_b32":
            setd(val(t[1]))
        elif op == "s_add_u32":
            r = val(t[1]) + val(t[2]); w.scc = r >> 32; setd(r)
        elif op == "s_addc_u32":
            r = val(t[1]) + val(t[2]) + w.scc; w.scc = r >> 32; setd(r)
        elif op == "s_sub_u32":
            r = val(t[1]) - val(t[2]); w.scc = 1 if r < 0 else 0; setd(r)
        elif op == "s_mul_i32":
            setd(val(t[1]) * val(t[2]))
        elif op == "s_mul_hi_u32":
            setd((val(t[1]) * val(t[2])) >> 32)
        elif op in ("s_lshl_b32", "s_lshr_b32", "s_and_b32", "s_or_b32", "s_xor_b32", "s_andn2_b32"):
            a, b = val(t[1]), val(t[2])
            r = {"s_lshl_b32": (a << (b & 31)) & M32, "s_lshr_b32": a >> (b & 31), "s_and_b32": a & b,
                 "s_or_b32": a | b, "s_xor_b32": a ^ b, "s_andn2_b32": a & ~b & M32}[op]
            setd(r); w.scc = int(r != 0)
        elif op == "s_lshl_b64":
            lo = reg_range(t[0])[0]
            src = reg_range(t[1])[0]
            v = int(S[src]) | (int(S[src + 1]) << 32)
            v = (v << val(t[2])) & ((1 << 64) - 1)
            S[lo], S[lo + 1] = v & M32, v >> 32
            w.scc = int(v != 0)
        elif op == "s_cselect_b32":
            setd(val(t[1]) if w.scc else val(t[2]))
        elif op.startswith("s_cmp_"):
            a, b = val(t[0]), val(t[1])
            w.scc = int({"eq_u32": a == b, "lt_u32": a < b, "ge_u32": a >= b, "eq_i32": a == b, "lg_u32": a != b,
                         "gt_u32": a > b}[op[6:]])
        elif op == "s_bitcmp1_b32":
            w.scc = (val(t[0]) >> val(t[1])) & 1
        elif op == "s_cbranch_scc0":
            if not w.scc:
                w.pc = self.labels[t[0]]
        elif op == "s_cbranch_scc1":
            if w.scc:
                w.pc = self.labels[t[0]]
        elif op == "s_branch":
            w.pc = self.labels[t[0]]
        else:
            raise RuntimeError("unsupported SALU " + op)
        return None

    def valu(self, w, op, t):
        V = w.v
        if op.endswith("_e64"):
            op = op[:-4]
        if op == "v_accvgpr_read_b32":
            V[d0(t)] = w.a[int(t[1][1:])].view(np.uint32)
            return None
        if op in ("v_permlane16_swap_b32", "v_permlane32_swap_b32"):
            # swap the odd rows (16 lanes) / upper half of vdst with the even rows / lower half of vsrc
            a, b = int(t[0][1:]), int(t[1][1:])
            va, vb = V[a].copy(), V[b].copy()
            for l in range(64):
                if op == "v_permlane32_swap_b32" and l >= 32:
                    va[l], vb[l - 32] = V[b][l - 32], V[a][l]
                elif op == "v_permlane16_swap_b32" and (l >> 4) & 1:
                    va[l], vb[l - 16] = V[b][l - 16], V[a][l]
            V[a], V[b] = va, vb
            return None
        if op == "v_readfirstlane_b32":
            w.s[int(t[0][1:])] = int(V[int(t[1][1:])][0])
            return None
        x = lambda i: self.vval(w, t[i])
        M = np.uint64(M32)
        if op == "v_lshrrev_b32":
            r = x(2) >> (x(1) & 31)
        elif op == "v_lshlrev_b32":
            r = (x(2) << (x(1) & 31)) & M
        elif op == "v_and_b32":
            r = x(1) & x(2)
        elif op == "v_xor_b32":
            r = x(1) ^ x(2)
        elif op == "v_add_u32":
            r = (x(1) + x(2)) & M
        elif op == "v_mov_b32":
            r = x(1)
        elif op == "v_lshl_add_u32":
            r = ((x(1) << (x(2) & 31)) + x(3)) & M
        elif op == "v_mad_u32_u24":
            r = ((x(1) & np.uint64(0xFFFFFF)) * (x(2) & np.uint64(0xFFFFFF)) + x(3)) & M
        elif op == "v_mul_lo_u32":
            r = (x(1) * x(2)) & M
        elif op in ("v_add_f32", "v_mul_f32", "v_fma_f32", "v_fmaak_f32", "v_rcp_f32", "v_exp_f32"):
            f = lambda i: self.fval(w, t[i])
            with np.errstate(all="ignore"):
                if op == "v_add_f32":
                    rf = f(1) + f(2)
                elif op == "v_mul_f32":
                    rf = f(1) * f(2)
                elif op == "v_fma_f32":
                    rf = (f(1).astype(np.float64) * f(2) + f(3)).astype(np.float32)
                elif op == "v_fmaak_f32":
                    rf = (f(1).astype(np.float64) * f(2) + f(3)).astype(np.float32)
                elif op == "v_rcp_f32":
                    rf = (np.float32(1.0) / f(1)).astype(np.float32)
                else:
                    rf = np.exp2(f(1)).astype(np.float32)
            r = rf.astype(np.float32).view(np.uint32).astype(np.uint64)
        elif op == "v_bfi_b32":
            r = (x(1) & x(2)) | (~x(1) & M & x(3))
        elif op == "v_subrev_u32":
            r = (x(2) - x(1)) & M
        elif op == "v_add3_u32":
            r = (x(1) + x(2) + x(3)) & M
        elif op == "v_bfe_u32":
            r = (x(1) >> (x(2) & 31)) & ((np.uint64(1) << (x(3) & 31)) - np.uint64(1))
        elif op == "v_cmp_gt_u32":
            assert t[0] == "vcc"
            w.vcc = x(1) > x(2)
            return None
        elif op == "v_cndmask_b32":
            assert t[3] == "vcc"
            r = np.where(w.vcc, x(2), x(1))
        elif op == "v_cvt_pk_bf16_f32":
            a = x(1).astype(np.uint32).view(np.float32)
            b = x(2).astype(np.uint32).view(np.float32)
            r = f32_to_bf16(a).astype(np.uint64) | (f32_to_bf16(b).astype(np.uint64) << np.uint64(16))
        else:
            raise RuntimeError("unsupported VALU " + op)
        V[int(t[0][1:])] = r.astype(np.uint32)
        return None

    def ds_read(self, w, op, t, mods):
        off = 0
        for m in mods:
            if m.startswith("offset:"):
                off = int(m[7:])
        dst, n = reg_range(t[0])
        addr = w.v[int(t[1][1:])].astype(np.int64) + off
        if op == "ds_read_b128":
            for l in range(64):
                a = int(addr[l])
                assert a % 16 == 0 and a + 16 <= self.lds_alloc, f"ds_read_b128 address {a}"
                w.v[dst:dst + 4, l] = self.lds[a:a + 16].view(np.uint32)
        elif op == "ds_read_b64_tr_b16":
            out = np.zeros((64, 4), dtype=np.uint16)
            for g in range(4):
                # lane 4q + p of the group supplies the address of row q, columns 4p..4p+3
                block = np.zeros((4, 16), dtype=np.uint16)
                for q in range(4):
                    for p in range(4):
                        a = int(addr[16 * g + 4 * q + p])
                        assert a % 8 == 0 and a + 8 <= self.lds_alloc, f"ds_read_b64_tr_b16 address {a}"
                        block[q, 4 * p:4 * p + 4] = self.lds[a:a + 8].view(np.uint16)
                for i in range(16):
                    out[16 * g + i] = block[:, i]
            w.v[dst:dst + 2] = out.view(np.uint32).reshape(64, 2).T
        else:
            raise RuntimeError("unsupported DS " + op)
        return None

    def srd(self, w, tok):
        b = reg_range(tok)[0]
        S = w.s
        base = int(S[b]) | ((int(S[b + 1]) & 0xFFFF) << 32)
        return base, int(S[b + 2])

    def buffer(self, w, op, t, mods):
        imm = 0
        for m in mods:
            if m.startswith("offset:"):
                imm = int(m[7:])
        assert "offen" in mods
        if op == "buffer_load_dwordx4" and "lds" in mods:
            voff = w.v[int(t[0][1:])].astype(np.int64)
            base, nr = self.srd(w, t[1])
            soff = self.sval(w, t[2])
            for l in range(64):
                o = int(voff[l]) + imm
                assert o + 16 <= nr, "DMA offset beyond num_records"
                data = self.mem.read(base + soff + o, 16)
                la = w.m0 + 16 * l
                assert la + 16 <= self.lds_alloc, f"LDS-DMA write at {la}"
                self.lds[la:la + 16] = data
            return None
        if op in ("buffer_load_dwordx4",):
            dst = reg_range(t[0])[0]
            voff = w.v[int(t[1][1:])].astype(np.int64)
            base, nr = self.srd(w, t[2])
            soff = self.sval(w, t[3])
            for l in range(64):
                data = self.mem.read(base + soff + int(voff[l]) + imm, 16).view(np.uint32)
                w.v[dst:dst + 4, l] = data
            return None
        if op in ("buffer_store_dword", "buffer_store_dwordx2", "buffer_store_dwordx4"):
            src, n = reg_range(t[0])
            n = {"buffer_store_dword": 1, "buffer_store_dwordx2": 2, "buffer_store_dwordx4": 4}[op]
            voff = w.v[int(t[1][1:])].astype(np.int64)
            base, nr = self.srd(w, t[2])
            soff = self.sval(w, t[3])
            for l in range(64):
                o = int(voff[l]) + imm
                assert o + 4 * n <= nr or nr == M32, "store beyond num_records"
                self.mem.write(base + soff + o, w.v[src:src + n, l].astype(np.uint32).view(np.uint8))
            return None
        raise RuntimeError("unsupported buffer op " + op)

    def mfma(self, w, t):
        dst = reg_range(t[0])[0]
        a0 = reg_range(t[1])[0]
        b0 = reg_range(t[2])[0]
        # A lane l: row l & 15, k 8 (l >> 4) + e (e = 0..7) in 4 VGPRs of 2 bf16
        av = w.v[a0:a0 + 4].T.copy().view(np.uint16).reshape(64, 8)
        bv = w.v[b0:b0 + 4].T.copy().view(np.uint16).reshape(64, 8)
        A = np.zeros((16, 32), dtype=np.float32)
        B = np.zeros((16, 32), dtype=np.float32)
        for l in range(64):
            A[l & 15, 8 * (l >> 4):8 * (l >> 4) + 8] = bf16_to_f32(av[l])
            B[l & 15, 8 * (l >> 4):8 * (l >> 4) + 8] = bf16_to_f32(bv[l])
        D = A @ B.T
        if t[3].strip() != "0":
            c0 = reg_range(t[3])[0]
            C = np.zeros((16, 16), dtype=np.float32)
            for l in range(64):
                for r in range(4):
                    C[4 * (l >> 4) + r, l & 15] = w.a[c0 + r, l]
            D = D + C
        for l in range(64):
            for r in range(4):
                w.a[dst + r, l] = D[4 * (l >> 4) + r, l & 15]
        return None


def d0(t):
    return int(t[0][1:])


def kernel_lds_bytes(asm_text, name):
    """the kernel descriptor's group_segment_fixed_size (the LDS the kernel allocates)"""
    m = re.search(r"\.amdhsa_kernel " + re.escape(name) + r"\s*\n\s*\.amdhsa_group_segment_fixed_size (\d+)", asm_text)
    return int(m.group(1)) if m else 131072


def run_kernel(asm_text, name, mem, kernarg, grid, wgs=None, lds_alloc=None):
    code, labels = parse_kernel(asm_text, name)
    if lds_alloc is None:
        lds_alloc = kernel_lds_bytes(asm_text, name)
    for wg in (range(grid) if wgs is None else wgs):
        Workgroup(code, labels, mem, kernarg, wg, lds_alloc=lds_alloc).run()


def selftest(asm_path):
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    text = open(asm_path).read()
    rng = np.random.default_rng(0)
    ok = True
    # ---- TN weight-grad kernel ----
    for (Ktot, M, N, splits) in [(512, 256, 256, 1), (1024, 512, 256, 2)]:
        A = rng.standard_normal((Ktot, M)).astype(np.float32)
        B = rng.standard_normal((Ktot, N)).astype(np.float32)
        Ab, Bb = f32_to_bf16(A), f32_to_bf16(B)
        mem = Memory()
        pa, pb = mem.alloc(Ab, "A"), mem.alloc(Bb, "B")
        pc = mem.alloc(np.full((splits, M, N), np.nan, dtype=np.float32), "C")
        units = (M // 256) * (N // 256) * splits
        ka = struct.pack("<6Q16i", pa, pb, pc, 0, 0, 0, M, N, Ktot // splits, M, N, N, N // 256, units, units, 0, 0, 0, 0, 0, 0, 0)
        run_kernel(text, "dalle_gemm_tn_wgrad", mem, ka, units)
        got = mem.get(pc, np.float32, (splits, M, N)).sum(0)
        ref = bf16_to_f32(Ab).T @ bf16_to_f32(Bb)
        err = float(np.abs(got - ref).max() / np.abs(ref).max())
        print(f"tn Ktot={Ktot} M={M} N={N} splits={splits}: max_rel_err {err:.2e}")
        ok &= err < 1e-4
    # ---- NT plain kernel (one tile per workgroup, grid = tiles) ----
    for (M, N, K) in [(256, 256, 256), (512, 256, 512)]:
        A = rng.standard_normal((M, K)).astype(np.float32)
        B = rng.standard_normal((N, K)).astype(np.float32)
        Ab, Bb = f32_to_bf16(A), f32_to_bf16(B)
        mem = Memory()
        pa, pb = mem.alloc(Ab, "A"), mem.alloc(Bb, "B")
        pc = mem.alloc(np.zeros((M, N), dtype=np.uint16), "C")
        nt = (M // 256) * (N // 256)
        grid = (nt + 7) // 8 * 8
        ka = struct.pack("<6Q16i", pa, pb, pc, 0, 0, 0, M, N, K, K, K, N, N // 256, nt, grid, 0, 0, 0, 0, 0, 0, 0)
        run_kernel(text, "dalle_gemm_nt_plain", mem, ka, grid)
        got = bf16_to_f32(mem.get(pc, np.uint16, (M, N)))
        ref = bf16_to_f32(Ab) @ bf16_to_f32(Bb).T
        err = float(np.abs(got - ref).max() / np.abs(ref).max())
        print(f"nt M={M} N={N} K={K}: max_rel_err {err:.2e}")
        ok &= err < 1e-2
    ok &= selftest_geglu(text)
    ok &= selftest_qkv(text, col=True) and selftest_qkv(text, col=False)
    return ok


def ff_in_perm(F):
    """interleaved row order of W1 for the geglu kernel: [value 4 | gate 4] blocks"""
    n = np.arange(2 * F)
    return 4 * (n >> 3) + (n & 3) + ((n >> 2) & 1) * F


def gelu_ref(x):
    from math import erf, sqrt
    return np.array([0.5 * v * (1 + erf(v / sqrt(2))) for v in x.ravel()], dtype=np.float64).reshape(x.shape)


def tile_of_wg(wg, grid, tiles_m, tiles_n):
    """(tm, tn) of the first tile of workgroup wg: the kernels' XCD map (grid a multiple of 8) and the grouped
    tile order of gen_gemm.tile_coords (8 tile rows per group, column-major inside)"""
    tile = (wg % 8) * (grid // 8) + wg // 8
    full = (tiles_m & ~7) * tiles_n
    if tile < full:
        g, w = divmod(tile, 8 * tiles_n)
        return 8 * g + w % 8, w // 8
    rem = tiles_m & 7
    w = tile - full
    return (tiles_m & ~7) + w % rem, w // rem


def selftest_qkv(text, col=True, T=257, S=16, H=4, B=2, K=1024, grid=8, wgs=None):
    rng = np.random.default_rng(2)
    I = S * S
    n = T + I - 1
    Tp = (T + 31) // 32 * 32
    Np = Tp + I
    M, N = B * n, 3 * H * 64
    h = f32_to_bf16(rng.standard_normal((M, K)).astype(np.float32))
    w = f32_to_bf16((rng.standard_normal((N, K)) * 0.03).astype(np.float32))
    cs = rng.uniform(-1, 1, (3, n + 1, 32, 2)).astype(np.float32)
    mem = Memory()
    ph, pw = mem.alloc(h, "h"), mem.alloc(w, "w")
    pq = mem.alloc(np.zeros((3, B * H, Np, 64), dtype=np.uint16), "qkv")
    pcs = mem.alloc(cs, "cs3")
    nt = (M // 256) * (N // 256)
    logS = S.bit_length() - 1
    ka = struct.pack("<6Q16i", ph, pw, pq, pcs, 0, 0, M, N, K, K, K, 0, N // 256, nt, grid, n, T, Tp, Np, H, logS, 0)
    run_kernel(text, "dalle_gemm_nt_qkv_col" if col else "dalle_gemm_nt_qkv_row", mem, ka, grid, wgs)
    got = mem.get(pq, np.uint16, (3, B * H, Np, 64))
    qkv = bf16_to_f32(f32_to_bf16(bf16_to_f32(h) @ bf16_to_f32(w).T)).reshape(B, n, 3, H, 32, 2)
    c, s_ = cs[:, :n, None, :, 0], cs[:, :n, None, :, 1]          # (3, n, 1, 32)
    x0, x1 = qkv[..., 0].transpose(2, 0, 1, 3, 4), qkv[..., 1].transpose(2, 0, 1, 3, 4)   # (3, B, n, H, 32)
    y0 = x0 * c[:, None] - x1 * s_[:, None]
    y1 = x1 * c[:, None] + x0 * s_[:, None]
    ref = np.zeros((3, B, H, Np, 64), dtype=np.float32)
    p = np.arange(n)
    k = p - T
    st = np.where(p < T, p, Tp + (((k % S) * S + k // S) if col else k))
    y = np.stack([y0, y1], -1).reshape(3, B, n, H, 64).transpose(0, 1, 3, 2, 4)   # (3, B, H, n, 64)
    ref[:, :, :, st] = y
    ref = ref.reshape(3, B * H, Np, 64)
    gotf = bf16_to_f32(got)
    if wgs is not None:     # only the tiles the chosen workgroups own (one tile each: grid >= tiles)
        errs = []
        for wg in wgs:
            tm, tn = tile_of_wg(wg, grid, M // 256, N // 256)
            rows = np.arange(tm * 256, tm * 256 + 256)
            b, pp = rows // n, rows % n
            for cc in range(tn * 256, tn * 256 + 256, 64):
                part, hh = cc // (H * 64), (cc % (H * 64)) // 64
                g_ = gotf[part, b * H + hh, st[pp]]
                r_ = ref[part, b * H + hh, st[pp]]
                errs.append(np.abs(g_ - r_).max())
        err = float(max(errs) / np.abs(ref).max())
        print(f"qkv col={col} wgs={wgs}: max_rel_err {err:.2e}")
        return err < 1.5e-2
    err = float(np.abs(gotf[:, :, st] - ref[:, :, st]).max() / np.abs(ref).max())
    print(f"qkv col={col} T={T} S={S} H={H} B={B}: max_rel_err {err:.2e}")
    return err < 1.5e-2


def gelu_and_grad_ref(x):
    from math import erf, exp, pi, sqrt
    xf = x.ravel().astype(np.float64)
    cdf = np.array([0.5 * (1 + erf(v / sqrt(2))) for v in xf])
    pdf = np.exp(-0.5 * xf * xf) / sqrt(2 * pi)
    return (xf * cdf).reshape(x.shape), (cdf + xf * pdf).reshape(x.shape)


def selftest_geglu_bwd(text, M=2560, F=256, K=1024, grid=8, wgs=(0, 1, 2)):
    """dh = GEGLU backward of du = bf16(dy W2) against the pre-activation a; part = 128-row column sums.
    M = 2560, F = 256: 10 tiles on 8 workgroups -- workgroups 0 and 1 walk two (the deferred path), 2 one."""
    rng = np.random.default_rng(3)
    dy = f32_to_bf16(rng.standard_normal((M, K)).astype(np.float32))
    w2t = f32_to_bf16((rng.standard_normal((F, K)) * 0.03).astype(np.float32))
    a = f32_to_bf16(rng.standard_normal((M, 2 * F)).astype(np.float32))
    mem = Memory()
    pa, pb = mem.alloc(dy, "dy"), mem.alloc(w2t, "w2t")
    pc = mem.alloc(np.zeros((M, 2 * F), dtype=np.uint16), "dh")
    ph = mem.alloc(a, "a")
    pp = mem.alloc(np.full((M // 128, 2 * F), np.nan, dtype=np.float32), "part")
    nt = (M // 256) * (F // 256)
    ka = struct.pack("<6Q16i", pa, pb, pc, ph, pp, 0, M, F, K, K, K, 2 * F, F // 256, nt, grid, F, 0, 0, 0, 0, 0, 0)
    run_kernel(text, "dalle_gemm_nt_geglu_bwd", mem, ka, grid, list(wgs), lds_alloc=163840)
    dh = bf16_to_f32(mem.get(pc, np.uint16, (M, 2 * F)))
    part = mem.get(pp, np.float32, (M // 128, 2 * F))
    du = bf16_to_f32(f32_to_bf16(bf16_to_f32(dy) @ bf16_to_f32(w2t).T)).astype(np.float64)
    af = bf16_to_f32(a).astype(np.float64)
    ge, gr = gelu_and_grad_ref(af[:, F:])
    ref = np.concatenate([du * ge, du * af[:, :F] * gr], 1)
    ok = True
    errs, perrs = [], []
    for wg in wgs:
        tile = (wg % 8) * (grid // 8) + wg // 8
        while tile < nt:
            tm, tn = tile_of_wg_id(tile, M // 256, F // 256)
            rows = slice(tm * 256, tm * 256 + 256)
            for c0 in (tn * 256, F + tn * 256):
                cols = slice(c0, c0 + 256)
                errs.append(np.abs(dh[rows, cols] - ref[rows, cols]).max())
                for blk in range(2):
                    rb = slice(tm * 256 + 128 * blk, tm * 256 + 128 * blk + 128)
                    psum = ref[rb, cols].sum(0)
                    perrs.append(np.abs(part[tm * 2 + blk, cols] - psum).max() / (np.abs(psum).max() + 1e-6))
            tile += grid
    err = float(max(errs) / np.abs(ref).max())
    perr = float(max(perrs))
    print(f"geglu_bwd M={M} F={F} wgs={list(wgs)}: dh max_rel_err {err:.2e}, column sums {perr:.2e}")
    return err < 1e-2 and perr < 2e-2


def tile_of_wg_id(tile, tiles_m, tiles_n):
    full = (tiles_m & ~7) * tiles_n
    if tile < full:
        g, w = divmod(tile, 8 * tiles_n)
        return 8 * g + w % 8, w // 8
    rem = tiles_m & 7
    w = tile - full
    return (tiles_m & ~7) + w % rem, w // rem


def selftest_geglu(text, M=2048, F=256, K=1024, grid=8, wgs=None, rows=None):
    """``wgs``: run only these workgroups and compare only output ``rows`` (the rows their tiles cover)"""
    rng = np.random.default_rng(1)
    x = f32_to_bf16(rng.standard_normal((M, K)).astype(np.float32))
    w1 = (rng.standard_normal((2 * F, K)) * 0.03).astype(np.float32)
    b1 = (rng.standard_normal(2 * F) * 0.1).astype(np.float32)
    perm = ff_in_perm(F)
    w1p = f32_to_bf16(w1[perm])
    b1p = b1[perm].astype(np.float32)
    mem = Memory()
    pa, pb = mem.alloc(x, "x"), mem.alloc(w1p, "w1p")
    pc = mem.alloc(np.zeros((M, 2 * F), dtype=np.uint16), "a")
    pbias = mem.alloc(b1p, "b1p")
    pu = mem.alloc(np.zeros((M, F), dtype=np.uint16), "u")
    nt = (M // 256) * (2 * F // 256)
    ka = struct.pack("<6Q16i", pa, pb, pc, pbias, pu, 0, M, 2 * F, K, K, K, 2 * F, 2 * F // 256, nt, grid, F, 0, 0, 0, 0, 0, 0)
    run_kernel(text, "dalle_gemm_nt_geglu", mem, ka, grid, wgs)
    sel = slice(None) if rows is None else rows
    a = bf16_to_f32(mem.get(pc, np.uint16, (M, 2 * F)))[sel]
    u = bf16_to_f32(mem.get(pu, np.uint16, (M, F)))[sel]
    a_ref = (bf16_to_f32(x) @ bf16_to_f32(f32_to_bf16(w1)).T + b1)[sel]
    err_a = float(np.abs(a - a_ref).max() / np.abs(a_ref).max())
    ab = a.astype(np.float64)
    u_ref = ab[:, :F] * gelu_ref(ab[:, F:])
    err_u = float(np.abs(u - u_ref).max() / np.abs(u_ref).max())
    print(f"geglu M={M} F={F} K={K}: a max_rel_err {err_a:.2e}, u (from the stored a) {err_u:.2e}")
    return err_a < 1e-2 and err_u < 1e-2


if __name__ == "__main__":
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "build", "asm",
                                                              "gemm_gfx950.s")
    sys.exit(0 if selftest(path) else 1)
