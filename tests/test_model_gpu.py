"""End-to-end HIP path vs the fp32 PyTorch reference (MI355X only)."""
import copy

import pytest
import torch

from dalle_amd.config import DALLEConfig, tiny
from dalle_amd.models.dalle import DALLE
from dalle_amd.optim import FlatArena, LAMB8bit

pytestmark = pytest.mark.gpu


def param_class(name: str) -> str:
    """parameter class of a DALLE state-dict name: sublayer kind + the module's own name, without layer indices
    (transformer.layers.layers.3.1.fn.fn.fn.net.0.weight -> ff.net.0.weight)"""
    import re

    m = re.match(r"transformer\.layers\.layers\.\d+\.(\d)\.(.*)$", name)          # sequential stack
    if m:
        kind = "attn." if m.group(1) == "0" else "ff."
    else:
        m = re.match(r"transformer\.layers\.blocks\.\d+\.([fg])\.net\.(.*)$", name)  # reversible stack
        if not m:
            return name
        kind = "attn." if m.group(1) == "f" else "ff."
    return kind + re.sub(r"^(fn\.)+", "", m.group(2))


# Per-class bounds on the relative gradient error (||g - g_ref|| / ||g_ref||, HIP bf16 path vs the fp32 CPU
# model), pinned at ~2x the worst value measured over every configuration below on the round-6 tree
# (profiles/r6_grad_err_pinned.txt: 0.0026-0.0074 for the layer parameters). The final LayerNorm bias of the
# reversible models is the sum over rows of a gradient that nearly cancels (measured up to 0.028): its own bound.
GRAD_BOUNDS = {"to_logits.0.bias": 0.06, "to_logits.1.bias": 0.02, "to_logits.0.weight": 0.008,
               "to_logits.1.weight": 0.012}
GRAD_BOUND_LAYER = 0.015


def check_grad_errors(errs: dict) -> None:
    bad = {k: v for k, v in errs.items() if v > GRAD_BOUNDS.get(k, GRAD_BOUND_LAYER)}
    assert not bad, bad


def grad_errors(m_hip, m_ref) -> dict:
    """worst relative gradient error (||g - g_ref|| / ||g_ref||) per parameter class"""
    ref = dict(m_ref.named_parameters())
    out = {}
    for name, p in m_hip.named_parameters():
        g, gr = p.grad.float().cpu(), ref[name].grad
        rel = ((g - gr).norm() / (gr.norm() + 1e-12)).item()
        c = param_class(name)
        out[c] = max(out.get(c, 0.0), rel)
    return out


def report(tag: str, errs: dict) -> None:
    import json

    print(f"GRAD_ERR {tag} " + json.dumps({k: round(v, 5) for k, v in sorted(errs.items())}))


def _cfg(reversible):
    c = tiny(reversible)
    types = ["axial_row", "axial_col", "conv_like", "full"]
    return DALLEConfig(**{**c.to_dict(), "depth": 4, "attn_types": types, "shared_attn_ids": [0, 1, 2, 3],
                          "shared_ff_ids": [0, 0, 1, 1]})


@pytest.mark.parametrize("reversible", [False, True])
def test_model_hip_matches_reference(cuda, reversible):
    torch.manual_seed(0)
    cfg = _cfg(reversible)
    m_ref = DALLE(cfg)
    # LayerScale 0.1 everywhere makes the branches matter
    m_hip = copy.deepcopy(m_ref).to(cuda)
    text = torch.randint(1, cfg.num_text_tokens, (2, cfg.text_seq_len))
    text[:, 50:] = 1
    img = torch.randint(0, cfg.num_image_tokens, (2, cfg.image_seq_len))
    loss_ref = m_ref(text, img, return_loss=True)
    loss_ref.backward()
    loss = m_hip(text.to(cuda), img.to(cuda), return_loss=True)
    loss.backward()
    assert abs(loss.item() - loss_ref.item()) < 2e-2 * abs(loss_ref.item())
    errs = grad_errors(m_hip, m_ref)
    report(f"tiny_rev{int(reversible)}", errs)
    check_grad_errors(errs)


def test_fused_lamb_matches_torch_path(cuda):
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(s, device=cuda)) for s in [(300, 400), (1000,), (70000,), (5, 4096)]]
    ps2 = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    arena = FlatArena(ps, device=cuda)
    kw = dict(lr=0.01, betas=(0.9, 0.96), eps=1e-6, weight_decay=0.045, clamp_value=10000.0, max_grad_norm=4.0)
    opt = LAMB8bit([{"params": ps[:2], "weight_decay": 0.045}, {"params": ps[2:], "weight_decay": 0.0}], arena=arena, **kw)
    opt2 = LAMB8bit([{"params": ps2[:2], "weight_decay": 0.045}, {"params": ps2[2:], "weight_decay": 0.0}], **kw)
    for it in range(3):
        for p, p2 in zip(ps, ps2):
            g = torch.randn_like(p)
            p.grad.copy_(g)
            p2.grad = g.clone()
        opt.step()
        opt2.step()
    assert opt._fused, "fused HIP engine must be active for arena parameters on GPU"
    for p, p2 in zip(ps, ps2):
        rel = ((p - p2).norm() / p2.norm()).item()
        assert rel < 1e-4, rel
    # 8-bit states: nearly identical indices
    st, st2 = opt.state[ps[0]], opt2.state[ps2[0]]
    assert st["state1"].dtype == torch.uint8
    agree = (st["state1"] == st2["state1"]).float().mean().item()
    assert agree > 0.99, agree
    assert torch.allclose(st["absmax1"], st2["absmax1"], rtol=1e-4)


@pytest.mark.parametrize("arena", [False, True])
def test_fused_reversible_matches_unfused(cuda, arena, monkeypatch):
    """The reversible stack over the fused sublayers (one recompute per block, hand-written
    backward, no autograd graph) vs the per-op reversible engine, both on the HIP kernels."""
    torch.manual_seed(0)
    cfg = _cfg(True)
    m1 = DALLE(cfg).to(cuda)
    m2 = copy.deepcopy(m1)
    text = torch.randint(1, cfg.num_text_tokens, (2, cfg.text_seq_len), device=cuda)
    img = torch.randint(0, cfg.num_image_tokens, (2, cfg.image_seq_len), device=cuda)
    grads = []
    import dalle_amd.ops as ops_mod

    for m, fused in ((m1, True), (m2, False)):
        monkeypatch.setattr(ops_mod, "FUSED_REVERSIBLE", fused)
        if arena:
            FlatArena(m.parameters(), device=cuda)
        loss = m(text, img, return_loss=True)
        loss.backward()
        grads.append((loss.item(), {n: p.grad.detach().float().clone() for n, p in m.named_parameters()}))
    (l1, g1), (l2, g2) = grads
    assert abs(l1 - l2) < 1e-3 * abs(l2)
    for name, g in g1.items():
        rel = ((g - g2[name]).norm() / (g2[name].norm() + 1e-8)).item()
        assert rel < 2e-2, (name, rel)


@pytest.mark.parametrize("budget_gb", [None, "0", "tiny"])
def test_reversible_auto_partial_storage(cuda, budget_gb, monkeypatch):
    """recompute="auto": the first blocks keep their activations while the HBM budget allows, the rest
    are rebuilt in backward -- loss bitwise equal, grads equal to the full-recompute path; a zero budget
    stores nothing and an unconstrained one (288 GB card, tiny model) stores every block."""
    from dalle_amd.ops import hip_ops

    torch.manual_seed(0)
    cfg = _cfg(True)
    m = DALLE(cfg).to(cuda)
    text = torch.randint(1, cfg.num_text_tokens, (2, cfg.text_seq_len), device=cuda)
    img = torch.randint(0, cfg.num_image_tokens, (2, cfg.image_seq_len), device=cuda)

    def run(policy):
        m.cfg.reversible_recompute = policy
        m.zero_grad(set_to_none=True)
        loss = m(text, img, return_loss=True)
        loss.backward()
        return loss.item(), {n: p.grad.float().clone() for n, p in m.named_parameters() if p.grad is not None}

    l_ref, g_ref = run(True)
    if budget_gb == "tiny":
        # room for about one and a half blocks: measure one block's bytes with an unconstrained run first
        monkeypatch.delenv("DALLE_AMD_REV_STORE_GB", raising=False)
        run("auto")
        per_block = hip_ops.REV_STATS["stored_bytes"] / max(hip_ops.REV_STATS["stored"], 1)
        monkeypatch.setenv("DALLE_AMD_REV_STORE_GB", str(3.5 * per_block / 2 ** 30))
    elif budget_gb is not None:
        monkeypatch.setenv("DALLE_AMD_REV_STORE_GB", budget_gb)
    l_auto, g_auto = run("auto")
    m.cfg.reversible_recompute = True
    stored, blocks = hip_ops.REV_STATS["stored"], hip_ops.REV_STATS["blocks"]
    if budget_gb is None:
        assert stored == blocks
    elif budget_gb == "0":
        assert stored == 0
    else:
        assert 0 < stored < blocks, (stored, blocks)
    assert l_auto == l_ref
    for n, g in g_ref.items():
        rel = ((g - g_auto[n]).norm() / (g.norm() + 1e-8)).item()
        assert rel < 2e-2, (n, rel)


def test_reversible_stored_activations_match_recompute(cuda):
    """reversible_recompute=False (activations kept from the forward) == the rebuild-in-backward path:
    same loss bitwise, gradients equal up to the reconstruction rounding of the recompute."""
    torch.manual_seed(0)
    cfg = _cfg(True)
    m = DALLE(cfg).to(cuda)
    text = torch.randint(1, cfg.num_text_tokens, (2, cfg.text_seq_len), device=cuda)
    img = torch.randint(0, cfg.num_image_tokens, (2, cfg.image_seq_len), device=cuda)
    grads, losses = [], []
    for recompute in (True, False):
        m.cfg.reversible_recompute = recompute
        m.zero_grad(set_to_none=True)
        loss = m(text, img, return_loss=True)
        loss.backward()
        losses.append(loss.item())
        grads.append({n: p.grad.float().clone() for n, p in m.named_parameters() if p.grad is not None})
    m.cfg.reversible_recompute = True
    assert losses[0] == losses[1]
    for n, g in grads[0].items():
        rel = ((g - grads[1][n]).norm() / (g.norm() + 1e-8)).item()
        assert rel < 2e-2, (n, rel)


def test_sequential_fused_stack_matches_per_sublayer(cuda, monkeypatch):
    """Non-reversible stack as one node with fused sublayer boundaries (ln_shift_fwd_res / ln_shift_bwd_sr)
    == the per-sublayer autograd nodes, with every gradient landing in the flat arena."""
    import dalle_amd.ops as ops_mod

    torch.manual_seed(0)
    cfg = _cfg(False)
    m = DALLE(cfg).to(cuda)
    arena = FlatArena(m.parameters(), device=cuda)
    text = torch.randint(1, cfg.num_text_tokens, (2, cfg.text_seq_len), device=cuda)
    img = torch.randint(0, cfg.num_image_tokens, (2, cfg.image_seq_len), device=cuda)
    grads, losses = [], []
    fused_stack = ops_mod.sequential_stack
    for fused in (1, 0):
        # the unfused arm: the stack declines and the model runs the per-sublayer nodes
        monkeypatch.setattr(ops_mod, "sequential_stack", fused_stack if fused else (lambda x, subs: None))
        arena.zero_grad()
        loss = m(text, img, return_loss=True)
        loss.backward()
        losses.append(loss.item())
        grads.append(arena.grad.clone())
    assert abs(losses[0] - losses[1]) <= 1e-5 * abs(losses[1])
    rel = ((grads[0] - grads[1]).norm() / grads[1].norm()).item()
    assert rel < 1e-3, rel
    # per parameter too (shared blocks accumulate from several sublayers)
    for p, o in zip(arena.params, arena.offsets):
        a, b = grads[0][o:o + p.numel()], grads[1][o:o + p.numel()]
        assert ((a - b).norm() / (b.norm() + 1e-12)).item() < 1e-2


def test_asm_gemm_step_matches_hipblaslt(cuda, monkeypatch):
    """The bench24 geometry (every plain projection tiles) with the plain products on the assembly GEMM vs on
    hipBLASLt: same loss and arena grads to bf16 rounding, and the assembly path really ran."""
    from dalle_amd.config import bench24
    from dalle_amd.ops import hip_ops

    torch.manual_seed(0)
    cfg = bench24()
    m = DALLE(cfg).to(cuda)
    arena = FlatArena(m.parameters(), device=cuda)
    m.grad_arena = arena
    text = torch.randint(1, cfg.num_text_tokens, (2, cfg.text_seq_len), device=cuda)
    img = torch.randint(0, cfg.num_image_tokens, (2, cfg.image_seq_len), device=cuda)
    out = {}
    for on in (True, False):
        monkeypatch.setattr(hip_ops, "ASM_GEMM", on)
        hip_ops.PATH_COUNTS.clear()
        arena.zero_grad()
        loss = m(text, img, return_loss=True)
        loss.backward()
        torch.cuda.synchronize()
        out[on] = (loss.item(), arena.grad.clone(), hip_ops.PATH_COUNTS.get("asm_gemm", 0))
    assert out[True][2] > 0 and out[False][2] == 0
    assert abs(out[True][0] - out[False][0]) <= 2e-3 * abs(out[False][0])
    rel = ((out[True][1] - out[False][1]).norm() / out[False][1].norm()).item()
    assert rel < 2e-2, rel


def _lamb_setup(cuda, seed=0):
    torch.manual_seed(seed)
    ps = [torch.nn.Parameter(torch.randn(s, device=cuda)) for s in [(300, 400), (1000,), (70000,), (5, 4096)]]
    arena = FlatArena(ps, device=cuda)
    kw = dict(lr=0.01, betas=(0.9, 0.96), eps=1e-6, weight_decay=0.045, clamp_value=10000.0, max_grad_norm=4.0)
    return ps, arena, LAMB8bit([{"params": ps[:2], "weight_decay": 0.045}, {"params": ps[2:], "weight_decay": 0.0}],
                               arena=arena, **kw)


def test_fused_lamb_state_is_8bit(cuda):
    """8-bit tensors hold uint8 moments + one fp32 absmax per 4096-block; fp32 moments exist only for the
    small tensors; no fp32 delta buffer (verdict r1 #8)."""
    ps, arena, opt = _lamb_setup(cuda)
    for p in ps:
        p.grad.normal_()
    opt.step()
    eng = opt._fused
    n8 = sum(p.numel() for p in ps if p.numel() >= 65536)
    n32 = sum(p.numel() for p in ps if p.numel() < 65536)
    ceil = lambda k: (k + 4095) // 4096 * 4096  # noqa: E731
    expect = 2 * sum(ceil(p.numel()) for p in ps if p.numel() >= 65536) + 8 * sum(ceil(p.numel()) // 4096 for p in ps if p.numel() >= 65536) \
        + 8 * sum(ceil(p.numel()) for p in ps if p.numel() < 65536)
    assert eng.state_bytes() == expect, (eng.state_bytes(), expect, n8, n32)
    assert not hasattr(eng, "delta")


def test_fused_lamb_restore_before_first_step(cuda):
    """state_dict -> a NEW optimizer -> load_state_dict BEFORE its first step -> step == uninterrupted run
    (the lazily created engine used to replace the restored moments with zeros)."""
    ps, arena, opt = _lamb_setup(cuda)
    torch.manual_seed(5)
    grads = [[torch.randn_like(p) for p in ps] for _ in range(3)]
    for it in range(2):
        for p, g in zip(ps, grads[it]):
            p.grad.copy_(g)
        opt.step()
    sd = copy.deepcopy(opt.state_dict())
    params_mid = arena.data.clone()
    for p, g in zip(ps, grads[2]):
        p.grad.copy_(g)
    opt.step()
    ref = arena.data.clone()

    ps2, arena2, opt2 = _lamb_setup(cuda, seed=1)
    arena2.data.copy_(params_mid)
    opt2.load_state_dict(sd)
    for p, g in zip(ps2, grads[2]):
        p.grad.copy_(g)
    opt2.step()
    assert opt2._fused
    assert torch.equal(arena2.data, ref)


@pytest.mark.parametrize("reversible,asm", [(False, False), (True, False), (False, True), (True, True)])
def test_reference_geometry_end_to_end(cuda, reversible, asm, monkeypatch):
    """The bench / reference geometry (d=1024, 16 heads, 256 text + 32x32 image tokens, the attention /
    sharing cycle of the recipe) with the flat arena attached, B=2 (M = 2560 = 10 x 256), so every fused
    path runs: QKV GEMM + rotary epilogue, FF dgrad + GEGLU-backward epilogue, the fused sequential /
    reversible stack. Loss and EVERY arena gradient vs the fp32 PyTorch model on the CPU."""
    from dalle_amd.config import DALLEConfig, reference_attn_types, reference_shared_ids
    from dalle_amd.data.synthetic import synthetic_batch
    from dalle_amd.ops import hip_ops

    # asm: the plain projections and the weight grads on the assembly GEMMs (token-major weight-grad inputs);
    # otherwise hipBLASLt with the token-contiguous transposed weight-grad inputs
    monkeypatch.setattr(hip_ops, "ASM_GEMM", asm)
    monkeypatch.setattr(hip_ops, "WGRAD_XT", not asm)
    monkeypatch.setattr(hip_ops, "WGRAD_GT", not asm)
    torch.manual_seed(0)
    cfg = DALLEConfig(depth=4, attn_types=reference_attn_types(4), shared_attn_ids=reference_shared_ids(4),
                      shared_ff_ids=reference_shared_ids(4), reversible=reversible)
    assert cfg.dim == 1024 and cfg.text_len == 257 and cfg.image_fmap_size == 32
    m_ref = DALLE(cfg)
    m_hip = copy.deepcopy(m_ref).to(cuda)
    arena = FlatArena(m_hip.parameters(), device=cuda)
    b = synthetic_batch(2, cfg.text_seq_len, cfg.image_seq_len, cfg.num_text_tokens, cfg.num_image_tokens,
                        torch.Generator().manual_seed(3))
    hip_ops.PATH_COUNTS.clear()
    loss = m_hip(b["input_ids"].to(cuda), b["image"].to(cuda), mask=b["attention_mask"].to(cuda), return_loss=True)
    loss.backward()
    torch.cuda.synchronize()
    stack = "reversible_stack" if reversible else "sequential_stack"
    for path in ("qkv_rope", "ff_dgrad_geglu", stack) + (("asm_gemm", "asm_wgrad") if asm else ("wgrad_xt",)):
        assert hip_ops.PATH_COUNTS.get(path, 0) > 0, (path, hip_ops.PATH_COUNTS)
    torch.set_num_threads(16)
    loss_ref = m_ref(b["input_ids"], b["image"], mask=b["attention_mask"], return_loss=True)
    loss_ref.backward()
    assert abs(loss.item() - loss_ref.item()) < 5e-3 * abs(loss_ref.item()), (loss.item(), loss_ref.item())
    errs = grad_errors(m_hip, m_ref)
    report(f"refgeom_rev{int(reversible)}_asm{int(asm)}", errs)
    check_grad_errors(errs)


@pytest.mark.parametrize("reversible", [False, True])
def test_1p3b_geometry_on_the_assembly_kernels(cuda, reversible):
    """BASELINE config 4's layer geometry (d_model 2048, 32 heads, 256 text + 32x32 image tokens, unshared
    layers) at depth 2, B = 2: QKV + rotary, FF-in + GEGLU, FF-dgrad + GEGLU backward and the tied head all run
    on the assembly kernels at K = 2048 (their successor K-steps 14..29 in the plain loop). Loss and every
    gradient vs the fp32 PyTorch model on the CPU."""
    from dalle_amd.config import large_1p3b, reference_attn_types
    from dalle_amd.data.synthetic import synthetic_batch
    from dalle_amd.ops import hip_ops

    torch.manual_seed(0)
    big = large_1p3b()
    cfg = DALLEConfig(**{**big.to_dict(), "depth": 2, "attn_types": reference_attn_types(2), "shared_attn_ids": [0, 1],
                         "shared_ff_ids": [0, 1], "reversible": reversible})
    assert cfg.dim == 2048 and cfg.heads == 32
    m_ref = DALLE(cfg)
    m_hip = copy.deepcopy(m_ref).to(cuda)
    FlatArena(m_hip.parameters(), device=cuda)
    b = synthetic_batch(2, cfg.text_seq_len, cfg.image_seq_len, cfg.num_text_tokens, cfg.num_image_tokens,
                        torch.Generator().manual_seed(3))
    hip_ops.PATH_COUNTS.clear()
    loss = m_hip(b["input_ids"].to(cuda), b["image"].to(cuda), mask=b["attention_mask"].to(cuda), return_loss=True)
    loss.backward()
    torch.cuda.synchronize()
    for path in ("asm_qkv_rope", "asm_ff_in_geglu", "asm_ff_dgrad_geglu", "asm_head", "asm_wgrad"):
        assert hip_ops.PATH_COUNTS.get(path, 0) > 0, (path, hip_ops.PATH_COUNTS)
    torch.set_num_threads(16)
    loss_ref = m_ref(b["input_ids"], b["image"], mask=b["attention_mask"], return_loss=True)
    loss_ref.backward()
    assert abs(loss.item() - loss_ref.item()) < 5e-3 * abs(loss_ref.item()), (loss.item(), loss_ref.item())
    errs = grad_errors(m_hip, m_ref)
    report(f"1p3b_rev{int(reversible)}", errs)
    check_grad_errors(errs)


def test_loss_trajectory_20_lamb_steps(cuda):
    """20 LAMB steps on the reference geometry (d 1024, 16 heads, 256 text + 32x32 image tokens, the recipe's
    attention / sharing cycle, depth 2): the HIP path (flat arena, fused LAMB) against the fp32 PyTorch model and
    the torch LAMB on the CPU, same init, same batches. Every step's loss stays within 0.1 % of the reference
    (measured max 7.3e-5 relative over the 20 steps, profiles/r6_grad_err_pinned.txt)."""
    from dalle_amd.config import reference_attn_types, reference_shared_ids
    from dalle_amd.data.synthetic import synthetic_batch

    torch.manual_seed(0)
    cfg = DALLEConfig(depth=2, attn_types=reference_attn_types(2), shared_attn_ids=reference_shared_ids(2),
                      shared_ff_ids=reference_shared_ids(2), reversible=False)
    m_ref = DALLE(cfg)
    m_hip = copy.deepcopy(m_ref).to(cuda)
    arena = FlatArena(m_hip.parameters(), device=cuda)
    kw = dict(lr=2e-3, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.0, max_grad_norm=4.0, optim_bits=32)
    opt_hip = LAMB8bit(m_hip.parameters(), arena=arena, **kw)
    opt_ref = LAMB8bit(m_ref.parameters(), **kw)
    gen = torch.Generator().manual_seed(5)
    batches = [synthetic_batch(2, cfg.text_seq_len, cfg.image_seq_len, cfg.num_text_tokens, cfg.num_image_tokens, gen)
               for _ in range(4)]
    torch.set_num_threads(16)
    dev = []
    for step in range(20):
        b = batches[step % 4]
        arena.zero_grad()
        loss = m_hip(b["input_ids"].to(cuda), b["image"].to(cuda), mask=b["attention_mask"].to(cuda), return_loss=True)
        loss.backward()
        opt_hip.step()
        opt_ref.zero_grad(set_to_none=True)
        loss_ref = m_ref(b["input_ids"], b["image"], mask=b["attention_mask"], return_loss=True)
        loss_ref.backward()
        opt_ref.step()
        dev.append(abs(loss.item() - loss_ref.item()) / abs(loss_ref.item()))
        print(f"step {step}: hip {loss.item():.5f} ref {loss_ref.item():.5f}")
    print("TRAJ max rel dev", max(dev))
    assert max(dev) < 1e-3, dev


@pytest.mark.parametrize("reversible", [False, True])
def test_grad_ready_handoff_reports_final_grads(cuda, reversible):
    """The fused stacks' backward hands every stack parameter to the data-parallel hook exactly once, and
    only when its arena grad is final (GradSync.attach all-reduces it right there, beside the rest of
    backward): the value seen at hand-off equals the value after backward, shared blocks included."""
    from dalle_amd.ops import hip_ops

    torch.manual_seed(0)
    cfg = _cfg(reversible)
    m = DALLE(cfg).to(cuda)
    arena = FlatArena(m.parameters(), device=cuda)
    text = torch.randint(1, cfg.num_text_tokens, (2, cfg.text_seq_len), device=cuda)
    img = torch.randint(0, cfg.num_image_tokens, (2, cfg.image_seq_len), device=cuda)
    seen = {}

    def record(params):
        for p in params:
            assert id(p) not in seen, "parameter handed over twice"
            seen[id(p)] = (p, p.grad.detach().clone())  # stream-ordered copy of the value at hand-off

    prev = hip_ops.set_grad_ready_hook(record)
    try:
        arena.zero_grad()
        m(text, img, return_loss=True).backward()
        torch.cuda.synchronize()
    finally:
        hip_ops.set_grad_ready_hook(prev)
    stack = {id(p) for n, p in m.named_parameters() if ".layers." in n or "transformer" in n}
    assert len(seen) > 0 and len(seen) >= len(stack) // 2, (len(seen), len(stack))
    for p, g_at in seen.values():
        assert torch.equal(g_at, p.grad), "grad changed after it was handed over"
    # the tied embedding / head and the final norm are not stack parameters: never handed over early
    assert id(m.to_logits[1].weight) not in seen


def test_head_fallback_for_wide_vocabulary_splits(cuda, monkeypatch):
    """Vocabulary splits wider than the CE kernel's LDS accumulator take the xent_fwd_bwd_ + PyTorch column
    sum path: same loss and gradients as the fused CE + bias-grad kernel."""
    from dalle_amd.ops import hip_ops

    torch.manual_seed(0)
    cfg = _cfg(False)
    m = DALLE(cfg).to(cuda)
    arena = FlatArena(m.parameters(), device=cuda)
    text = torch.randint(1, cfg.num_text_tokens, (2, cfg.text_seq_len), device=cuda)
    img = torch.randint(0, cfg.num_image_tokens, (2, cfg.image_seq_len), device=cuda)
    out = []
    for maxv in (hip_ops.XENT_COLSUM_MAXV, 0):
        monkeypatch.setattr(hip_ops, "XENT_COLSUM_MAXV", maxv)
        arena.zero_grad()
        loss = m(text, img, return_loss=True)
        loss.backward()
        out.append((loss.item(), arena.grad.clone()))
    assert abs(out[0][0] - out[1][0]) <= 1e-6 * abs(out[0][0])
    assert torch.allclose(out[0][1], out[1][1], rtol=1e-4, atol=1e-7)
