"""The assembly kernels build on a GPU-less host: gen_gemm.py emits gfx950 assembly that clang assembles and
ld.lld links into a code object whose kernel descriptors carry the register / LDS budget the schedule assumes
(one 256-thread workgroup per CU: 512 VGPR+AGPR, 128 KB LDS); the generator never emits a scalar-memory store."""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


@pytest.mark.skipif(not os.path.exists(os.path.join(LLVM, "clang")), reason="ROCm LLVM not installed")
def test_asm_gemm_builds(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "csrc", "asm"))
    import gen_gemm

    s = tmp_path / "g.s"
    gen_gemm.main(str(s))
    text = s.read_text()
    assert not re.search(r"\bs_(store|atomic|dcache|buffer_store|scratch_store)", text)
    o, co = tmp_path / "g.o", tmp_path / "g.hsaco"
    subprocess.run([os.path.join(LLVM, "clang"), "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c",
                    str(s), "-o", str(o)], check=True)
    subprocess.run([os.path.join(LLVM, "ld.lld"), "-shared", str(o), "-o", str(co)], check=True)
    notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", str(co)], capture_output=True, text=True,
                           check=True).stdout
    for name, _, _ in gen_gemm.KERNELS:
        assert f".name:           {name}" in notes
    assert notes.count(".vgpr_count:     512") == len(gen_gemm.KERNELS)
    for name, _, _ in gen_gemm.KERNELS:   # two 64 KB operand stages; the GEGLU backward also its 32 KB stash
        lds = gen_gemm.LDS_BYTES.get(name, 131072)
        assert lds <= 160 * 1024
    big = sum(1 for name, _, _ in gen_gemm.KERNELS if name in gen_gemm.LDS_BYTES)
    assert notes.count(".group_segment_fixed_size: 131072") == len(gen_gemm.KERNELS) - big
    assert notes.count(".group_segment_fixed_size: 163840") == big
    # per K-step and wave: 128 MFMAs, 16 LDS-DMA pieces, 32 fragment reads; the plain kernel's loop body has 2
    # barriers (stage released, next step landed), the fused kernels' 3 (A image released, B image released,
    # next step landed)
    for name, nbar in (("dalle_gemm_nt_plain", 2), ("dalle_gemm_nt_geglu", 3)):
        body = text.split(f"{name}_kloop:")[1].split("s_cbranch_scc0")[0]
        assert body.count("v_mfma_f32_16x16x32_bf16") == 128
        assert body.count(" lds") == 16 and body.count("ds_read_b128") == 32 and body.count("s_barrier") == nbar
        assert "s_nop" not in body   # every wait state of the loop is an MFMA


def test_kernel_generation_is_order_independent(tmp_path):
    """Every kernel is generated from the default schedule knobs: the production set emitted in its own order
    and in the reverse order with every diagnostic variant interleaved gives byte-identical production code."""
    sys.path.insert(0, os.path.join(ROOT, "csrc", "asm"))
    import gen_gemm

    fwd, rev = tmp_path / "fwd.s", tmp_path / "rev.s"
    gen_gemm.main(str(fwd))
    mix = []
    for i, k in enumerate(gen_gemm.KERNELS):
        mix += gen_gemm.DIAG_KERNELS[3 * i:3 * i + 3] + [k]
    mix += gen_gemm.DIAG_KERNELS[3 * len(gen_gemm.KERNELS):]
    gen_gemm.main(str(rev), kernels=list(reversed(mix)))
    a, b = fwd.read_text(), rev.read_text()

    def body(text, name):
        i = text.index(f"{name}:\n")
        return text[i:text.index(f"\t.size\t{name}", i)]

    for name, _, _ in gen_gemm.KERNELS:
        assert body(a, name) == body(b, name), name


def test_default_build_skips_diagnostic_kernels():
    src = open(os.path.join(ROOT, "csrc", "asm", "build_asm.py")).read()
    assert 'os.environ.get("DALLE_AMD_BUILD_DIAG", "0") != "1"' in src


def test_fragment_reads_are_bank_conflict_free():
    """The operand image layout (row-major 128-B rows, chunk c of row r at position c ^ ((r >> 1) & 7)) read as
    gen_gemm.lane_setup / frag_reads address it: under the ds_read_b128 lane grouping (4 groups of 16 lanes,
    MI355X_MICROARCH.md LDS table) every group touches 16 distinct 16-byte bank slots, for every fragment."""
    g0 = list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28))
    g1 = list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))
    groups = [g0, g1, [l + 32 for l in g0], [l + 32 for l in g1]]
    for h in (0, 1):
        for f in range(8):
            addr = {}
            for lane in range(64):
                p, kg = lane & 15, lane >> 4
                row = 16 * f + p
                addr[lane] = row * 128 + (((4 * h + kg) ^ ((row >> 1) & 7)) * 16)
            for g in groups:
                assert len({(addr[l] // 16) % 16 for l in g}) == 16, (h, f)
    # the DMA writes what the reads expect: lane t of instruction (rows 8 d ..) loads global chunk
    # c' ^ (4 (d & 1) + (r' >> 1)) into position c' of image row 8 d + r'
    for d in range(32):
        for t in range(64):
            r_img, pos = 8 * d + (t >> 3), t & 7
            chunk = pos ^ (4 * (d & 1) + ((t >> 3) >> 1))
            assert pos == chunk ^ ((r_img >> 1) & 7)


@pytest.mark.skipif(not os.path.exists(os.path.join(LLVM, "clang")), reason="ROCm LLVM not installed")
def test_kernels_on_the_emulator(tmp_path):
    """csrc/asm/emu.py runs the generated NT and TN kernels instruction by instruction on one small shape each,
    bounds-checking every global / LDS access, and compares with numpy (it caught the TN kernel's unmasked
    lane fields -- an out-of-range store -- before a second GPU run)."""
    sys.path.insert(0, os.path.join(ROOT, "csrc", "asm"))
    import struct

    import numpy as np

    import emu
    import gen_gemm

    s = tmp_path / "g.s"
    gen_gemm.main(str(s))
    text = s.read_text()
    rng = np.random.default_rng(0)
    Ktot, M, N = 512, 256, 256
    Ab = emu.f32_to_bf16(rng.standard_normal((Ktot, M)).astype(np.float32))
    Bb = emu.f32_to_bf16(rng.standard_normal((Ktot, N)).astype(np.float32))
    mem = emu.Memory()
    pa, pb = mem.alloc(Ab, "A"), mem.alloc(Bb, "B")
    pc = mem.alloc(np.zeros((M, N), dtype=np.float32), "C")
    ka = struct.pack("<6Q16i", pa, pb, pc, 0, 0, 0, M, N, Ktot, M, N, N, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0)
    emu.run_kernel(text, "dalle_gemm_tn_wgrad", mem, ka, 1)
    ref = emu.bf16_to_f32(Ab).T @ emu.bf16_to_f32(Bb)
    got = mem.get(pc, np.float32, (M, N))
    assert np.abs(got - ref).max() / np.abs(ref).max() < 1e-4
    K = 256
    Ab = emu.f32_to_bf16(rng.standard_normal((M, K)).astype(np.float32))
    Bb = emu.f32_to_bf16(rng.standard_normal((N, K)).astype(np.float32))
    mem = emu.Memory()
    pa, pb = mem.alloc(Ab, "A"), mem.alloc(Bb, "B")
    pc = mem.alloc(np.zeros((M, N), dtype=np.uint16), "C")
    ka = struct.pack("<6Q16i", pa, pb, pc, 0, 0, 0, M, N, K, K, K, N, 1, 1, 8, 0, 0, 0, 0, 0, 0, 0)
    emu.run_kernel(text, "dalle_gemm_nt_plain", mem, ka, 8)
    ref = emu.bf16_to_f32(Ab) @ emu.bf16_to_f32(Bb).T
    got = emu.bf16_to_f32(mem.get(pc, np.uint16, (M, N)))
    assert np.abs(got - ref).max() / np.abs(ref).max() < 1e-2


def test_fused_epilogue_kernels_on_the_emulator(tmp_path):
    """The FF-out dgrad + GEGLU backward kernel on the emulator: one workgroup walking two tiles, so both the
    deferred path (row-groups at the boundary, in VGPRs and in LDS, processed under the successor's K-steps,
    permlane-folded column sums) and the final path run; and the QKV + rotary kernel's first workgroup."""
    sys.path.insert(0, os.path.join(ROOT, "csrc", "asm"))
    import emu
    import gen_gemm

    s = tmp_path / "g.s"
    gen_gemm.main(str(s))
    text = s.read_text()
    assert emu.selftest_geglu_bwd(text, M=2560, F=256, grid=8, wgs=(0,))
    assert emu.selftest_qkv(text, col=True, T=257, S=16, H=4, B=2, grid=8, wgs=[0])


def test_fused_kernels_at_k2048_on_the_emulator(tmp_path):
    """The fused kernels at K = 2048 (the ~1.3B config's d_model): the successor tile's unrolled K-steps 0..13
    hand over to the ordinary K-loop for steps 14..29 before the tail -- one workgroup walking two or three
    tiles of the GEGLU backward, FF-in + GEGLU and QKV + rotary kernels."""
    sys.path.insert(0, os.path.join(ROOT, "csrc", "asm"))
    import emu
    import gen_gemm

    s = tmp_path / "g.s"
    gen_gemm.main(str(s))
    text = s.read_text()
    assert emu.selftest_geglu_bwd(text, M=2560, F=256, K=2048, grid=8, wgs=(0,))
    assert emu.selftest_geglu(text, M=4096, F=256, K=2048, grid=8, wgs=[0], rows=slice(0, 256))
    assert emu.selftest_qkv(text, col=False, T=257, S=16, H=4, B=4, K=2048, grid=8, wgs=[0])


def test_plain_kernel_deferred_paths_on_the_emulator(tmp_path):
    """Two tiles per workgroup through the plain and bias kernels: K = 1024 (stores spread over the successor's
    K-steps 0..12) and K = 512 (over 0..3)."""
    sys.path.insert(0, os.path.join(ROOT, "csrc", "asm"))
    import struct

    import numpy as np

    import emu
    import gen_gemm

    s = tmp_path / "g.s"
    gen_gemm.main(str(s))
    text = s.read_text()
    for name, K, bias in (("dalle_gemm_nt_bias", 1024, True), ("dalle_gemm_nt_plain", 512, False)):
        rng = np.random.default_rng(K)
        M, N = 2560, 256
        A = emu.f32_to_bf16(rng.standard_normal((M, K)).astype(np.float32))
        B = emu.f32_to_bf16(rng.standard_normal((N, K)).astype(np.float32))
        b = rng.standard_normal(N).astype(np.float32)
        mem = emu.Memory()
        pa, pb = mem.alloc(A, "A"), mem.alloc(B, "B")
        pc = mem.alloc(np.zeros((M, N), dtype=np.uint16), "C")
        pbias = mem.alloc(b, "bias")
        nt, grid = (M // 256) * (N // 256), 8
        ka = struct.pack("<6Q16i", pa, pb, pc, pbias if bias else 0, 0, 0, M, N, K, K, K, N, N // 256, nt, grid,
                         0, 0, 0, 0, 0, 0, 0)
        emu.run_kernel(text, name, mem, ka, grid, [0])
        got = emu.bf16_to_f32(mem.get(pc, np.uint16, (M, N)))
        ref = emu.bf16_to_f32(A) @ emu.bf16_to_f32(B).T + (b if bias else 0)
        rows = list(range(0, 256)) + list(range(8 * 256, 9 * 256))     # workgroup 0: tiles 0 and 8
        assert np.abs(got[rows] - ref[rows]).max() / np.abs(ref).max() < 1e-2
