"""Optimizer tests (SURVEY §4 tier 3): dynamic maps, blockwise quantisation, 8-bit LAMB."""
import copy

import numpy as np
import pytest
import torch

from dalle_amd.optim import FlatArena, LAMB8bit, LambWithGradientClipping, get_linear_schedule_with_warmup
from dalle_amd.optim import quant


def _numpy_dynamic_map(signed):
    # independent NumPy re-derivation of bitsandbytes.functional.create_dynamic_map(signed, n=7)
    data = []
    for i in range(7):
        items = 2 ** i + 1 if signed else 2 ** (i + 1) + 1
        b = np.linspace(0.1, 1, items, dtype=np.float32)
        means = (b[:-1] + b[1:]) / 2.0
        data += list((10 ** (-6 + i)) * means)
        if signed:
            data += list(-(10 ** (-6 + i)) * means)
    data += [0.0, 1.0]
    return np.sort(np.array(data, dtype=np.float32))


@pytest.mark.parametrize("signed", [True, False])
def test_dynamic_map(signed):
    m = quant.dynamic_map(signed).numpy()
    assert m.shape == (256,)
    assert np.all(np.diff(m) >= 0)
    assert np.allclose(m, _numpy_dynamic_map(signed), rtol=1e-6, atol=1e-12)
    assert m.max() == 1.0
    assert (m.min() < -0.99) if signed else (m.min() == 0.0)


def test_quantize_roundtrip_and_nearest():
    torch.manual_seed(0)
    x = torch.randn(3 * 4096 + 123) * torch.logspace(-4, 0, 3 * 4096 + 123)
    code = quant.dynamic_map(True)
    q, absmax = quant.quantize_blockwise(x, code)
    assert q.dtype == torch.uint8 and absmax.shape == (4,)
    y = quant.dequantize_blockwise(q, absmax, code)
    # nearest-entry property: no other code gives a smaller error
    normed = x / absmax.repeat_interleave(4096)[: x.numel()]
    err_best = (code[None, :] - normed[:, None]).abs().min(dim=1).values
    err = (code[q.long()] - normed).abs()
    assert torch.allclose(err, err_best, atol=1e-7)
    rel = ((y - x).norm() / x.norm()).item()
    assert rel < 0.05


def test_lamb_8bit_close_to_fp32():
    torch.manual_seed(0)
    w0 = torch.randn(256, 512) * 0.02
    p8, p32 = torch.nn.Parameter(w0.clone()), torch.nn.Parameter(w0.clone())
    kw = dict(lr=0.01, betas=(0.9, 0.96), eps=1e-6, weight_decay=0.045, clamp_value=10000.0, max_grad_norm=4.0)
    o8 = LAMB8bit([p8], **kw)
    o32 = LambWithGradientClipping([p32], **kw)
    for _ in range(5):
        g = torch.randn_like(w0)
        p8.grad, p32.grad = g.clone(), g.clone()
        o8.step()
        o32.step()
    st = o8.state[p8]
    assert st["state1"].dtype == torch.uint8 and st["state2"].dtype == torch.uint8
    assert st["absmax1"].shape == (32,)
    assert o32.state[p32]["state1"].dtype == torch.float32
    d8, d32 = p8 - w0, p32 - w0
    assert ((d8 - d32).norm() / d32.norm()).item() < 0.1
    for k in ("step", "state1", "state2", "qmap1", "qmap2", "absmax1", "absmax2", "weight_norm", "step_norm", "trust_ratio"):
        assert k in st


def test_lamb_small_tensor_fp32_states_and_trust_ratio():
    p = torch.nn.Parameter(torch.ones(1000))
    opt = LAMB8bit([p], lr=0.1, weight_decay=0.0, clamp_value=10.0)
    p.grad = torch.ones(1000)
    opt.step()
    st = opt.state[p]
    assert st["state1"].dtype == torch.float32  # numel < min_8bit_size
    # m = 0.1, v = 0.001 -> delta = 0.1/(sqrt(0.001)+eps) ~ 3.162 per elem; |p| = 31.6 clamps to 10
    d = 0.1 / (0.001 ** 0.5 + 1e-6)
    trust = 10.0 / (d * 1000 ** 0.5)
    assert torch.allclose(p.data, torch.full((1000,), 1 - 0.1 * trust * d), atol=1e-5)


def test_lamb_validation_errors():
    p = torch.nn.Parameter(torch.zeros(3))
    with pytest.raises(ValueError):
        LAMB8bit([p], lr=-1)
    with pytest.raises(ValueError):
        LAMB8bit([p], betas=(1.0, 0.9))
    with pytest.raises(ValueError):
        LAMB8bit([p], weight_decay=-1)


def test_flat_arena_views_and_grad_accumulation():
    lin = torch.nn.Linear(10, 7)
    arena = FlatArena(lin.parameters())
    assert arena.numel == 2 * 4096
    assert lin.weight.data_ptr() == arena.data.data_ptr()
    lin(torch.randn(3, 10)).sum().backward()
    assert lin.weight.grad.data_ptr() == arena.grad.data_ptr()
    g1 = arena.grad.clone()
    lin(torch.randn(3, 10)).sum().backward()  # accumulates in place
    assert not torch.equal(g1, arena.grad)
    arena.zero_grad()
    assert arena.grad.abs().sum() == 0
    assert arena.block_tensor.tolist() == [0, 1]


def test_linear_schedule():
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=1.0)
    sch = get_linear_schedule_with_warmup(opt, 10, 100)
    lrs = []
    for _ in range(100):
        lrs.append(opt.param_groups[0]["lr"])
        opt.step()
        sch.step()
    assert lrs[0] == 0.0 and abs(lrs[10] - 1.0) < 1e-9 and abs(lrs[55] - 0.5) < 1e-9


def test_state_dict_roundtrip():
    torch.manual_seed(0)
    p = torch.nn.Parameter(torch.randn(100, 1000))
    opt = LAMB8bit([p], lr=0.01)
    p.grad = torch.randn_like(p)
    opt.step()
    sd = copy.deepcopy(opt.state_dict())  # state_dict() returns live references
    p2 = torch.nn.Parameter(p.detach().clone())
    opt2 = LAMB8bit([p2], lr=0.01)
    opt2.load_state_dict(sd)
    g = torch.randn_like(p)
    p.grad, p2.grad = g.clone(), g.clone()
    opt.step()
    opt2.step()
    assert torch.allclose(p, p2)


def test_monitor_summary_matches_reference_aggregation():
    """Aux-peer aggregation (dalle_amd.utils.monitor.summarize): mean loss over all mini-steps, summed
    samples and samples/s, alive peers = records."""
    from types import SimpleNamespace as R

    from dalle_amd.utils.monitor import summarize

    recs = [R(step=7, loss=6.0, mini_steps=3, samples_accumulated=12, samples_per_second=10.0),
            R(step=7, loss=2.0, mini_steps=1, samples_accumulated=4, samples_per_second=2.5)]
    s = summarize(recs)
    assert s.step == 7 and s.alive_peers == 2 and s.samples == 16
    assert abs(s.loss - 2.0) < 1e-12 and abs(s.performance - 12.5) < 1e-12
    assert s.as_record()["alive peers"] == 2
    assert summarize([]) is None


def test_preprocess_batch_filters_and_decodes():
    import numpy as np

    from data import preprocess_batch

    class Tok:
        def __call__(self, texts, add_special_tokens, max_length, truncation):
            assert add_special_tokens is False and truncation
            ids = [[len(t)] * min(len(t), max_length) for t in texts]
            return {"input_ids": ids, "attention_mask": [[1] * len(i) for i in ids]}

    code = np.arange(4, dtype=np.int16).tobytes()
    batch = {"caption": ["a cat", "no", None, "a wide one", "nsfw", "ok caption"],
             "NSFW": ["UNLIKELY", "UNLIKELY", "UNLIKELY", "UNLIKELY", "LIKELY", "UNLIKELY"],
             "original_width": [100, 100, 100, 500, 100, 100], "original_height": [100, 100, 100, 100, 100, 200],
             "code": [code] * 6}
    out = preprocess_batch(batch, Tok(), 3)
    assert out["input_ids"] == [[5, 5, 5], [10, 10, 10]]  # "a cat", "ok caption" (aspect exactly 2 is kept)
    assert len(out["image"]) == 2 and out["image"][0].dtype == np.int64 and list(out["image"][1]) == [0, 1, 2, 3]
    empty = preprocess_batch({k: v[1:3] for k, v in batch.items()}, Tok(), 3)
    assert empty == {"input_ids": [], "attention_mask": [], "image": []}


def test_local_and_datasets_streaming_sources(tmp_path):
    """Parquet shards in the laion_100m_vqgan_f8 column layout: the local directory reader (streamed
    record batches) and the `datasets` streaming source (`parquet:<glob>`, the reference's
    load_dataset(..., streaming=True) path) yield the same filtered, tokenised examples."""
    import numpy as np
    import pyarrow as pa
    import pyarrow.parquet as pq

    from data import make_dataset

    class Tok:
        def __call__(self, texts, add_special_tokens, max_length, truncation):
            ids = [[len(t) % 7 + 1] * min(len(t), max_length) for t in texts]
            return {"input_ids": ids, "attention_mask": [[1] * len(i) for i in ids]}

    rng = np.random.default_rng(0)
    for shard in range(2):
        n = 40
        caps = [f"caption number {shard}-{i}" if i % 5 else "no" for i in range(n)]
        tbl = pa.table({"caption": caps, "NSFW": ["UNLIKELY" if i % 7 else "LIKELY" for i in range(n)],
                        "original_width": [256] * n, "original_height": [256] * n,
                        "code": [rng.integers(0, 8192, 16, dtype=np.int16).tobytes() for _ in range(n)]})
        pq.write_table(tbl, tmp_path / f"part-{shard}.parquet")
    kw = dict(shuffle_buffer_size=1, shuffle_seed=0, preprocessing_batch_size=16, max_sequence_length=8)
    local = list(make_dataset(Tok(), dataset_path=str(tmp_path), **kw))
    kept = sum(1 for s in range(2) for i in range(40) if i % 5 and i % 7)
    assert len(local) == kept
    assert all(ex["image"].dtype == torch.int64 and ex["image"].shape == (16,) for ex in local)
    streamed = list(make_dataset(Tok(), dataset_path=f"parquet:{tmp_path}/*.parquet", **kw))
    assert len(streamed) == kept
    key = lambda ex: tuple(ex["image"].tolist())  # noqa: E731
    assert sorted(map(key, streamed)) == sorted(map(key, local))


def test_delegating_optimizer():
    from dalle_amd.optim.wrapper import OptimizerWrapper

    class Counting(OptimizerWrapper):
        _own = ("inner", "steps")

        def __init__(self, inner):
            super().__init__(inner)
            self.steps = 0

        def step(self, closure=None):
            self.steps += 1
            return super().step(closure)

    p = torch.nn.Parameter(torch.ones(3))
    opt = Counting(torch.optim.SGD([p], lr=0.5))
    p.grad = torch.ones(3)
    opt.step()
    assert opt.steps == 1 and torch.allclose(p.detach(), torch.full((3,), 0.5))
    assert opt.param_groups[0]["lr"] == 0.5 and opt.defaults["lr"] == 0.5
    opt.param_groups[0]["lr"] = 0.1  # protocol objects are the inner optimizer's
    assert opt.inner.param_groups[0]["lr"] == 0.1
    sd = opt.state_dict()
    opt.load_state_dict(sd)
    opt.zero_grad()
    assert p.grad is None
    assert "Counting(" in repr(opt)


def _offload_vs_plain(dev, dtype=torch.float32, steps=4):
    from dalle_amd.optim.wrapper import HostOffloadOptimizer

    torch.manual_seed(0)
    init = [torch.randn(7, 5), torch.randn(11), torch.randn(3, 2, 2)]
    grads = [[torch.randn_like(t) for t in init] for _ in range(steps)]
    a = [torch.nn.Parameter(t.clone().to(dev, dtype)) for t in init]
    b = [torch.nn.Parameter(t.clone().to(dev, dtype)) for t in init]
    plain = torch.optim.Adam([{"params": a[:2]}, {"params": a[2:], "lr": 3e-3}], lr=1e-2, weight_decay=0.1)
    off = HostOffloadOptimizer(torch.optim.Adam([{"params": b[:2]}, {"params": b[2:], "lr": 3e-3}], lr=1e-2,
                                                weight_decay=0.1))
    for gs in grads:
        for ps, opt in ((a, plain), (b, off)):
            for p, g in zip(ps, gs):
                p.grad = g.to(dev, dtype)
            opt.step()
            opt.zero_grad()
    return a, b, off


def test_host_offload_optimizer_matches_plain_step():
    a, b, off = _offload_vs_plain("cpu")
    for x, y in zip(a, b):
        torch.testing.assert_close(x, y, rtol=1e-6, atol=1e-7)
    # the state lives with the host copies, keyed by the inner optimizer's parameter order
    st = off.state_dict()
    assert len(st["state"]) == 3 and st["state"][0]["exp_avg"].shape == (7, 5)
    assert all(v["exp_avg"].device.type == "cpu" for v in off.inner.state.values())
    off.load_state_dict(st)
    assert off.param_groups[1]["lr"] == 3e-3 and off.param_groups[0]["params"][0] is b[0]
    with pytest.raises(ValueError):
        off.step(closure=lambda: 0.0)


def test_collaborative_optimizer_offloads_a_prebuilt_optimizer():
    """A built optimizer (no factory) + offload_device: the collaborative optimizer steps it through
    HostOffloadOptimizer (world 1: no process group needed)."""
    from dalle_amd.optim.wrapper import HostOffloadOptimizer
    from dalle_amd.parallel.optimizer import CollaborativeOptimizer

    p = torch.nn.Parameter(torch.ones(4))
    opt = CollaborativeOptimizer(run_id="off", params=[p], optimizer=torch.optim.SGD([p], lr=0.5),
                                 target_batch_size=1, batch_size_per_step=1, offload_device="cpu",
                                 tracker_mode="static")
    assert isinstance(opt.state_averager.optimizer, HostOffloadOptimizer)
    p.grad = torch.ones(4)
    opt.step()
    assert torch.allclose(p.detach(), torch.full((4,), 0.5)) and opt.local_epoch == 1


class _FakeDevice:
    """A device timeline that runs each step in `dev_ms` while the host enqueues every `host_ms`."""

    def __init__(self, dev_ms):
        self.dev_ms, self.t_dev, self.t_host = dev_ms, 0.0, 0.0

    def record(self):
        dev = self
        self.t_dev = max(self.t_dev, self.t_host) + self.dev_ms  # the step's kernels finish at t_dev
        done_at = self.t_dev

        class Ev:
            t = done_at

            def query(self_):
                return dev.t_host >= self_.t

            def elapsed_time(self_, other):
                return other.t - self_.t

            def synchronize(self_):
                dev.t_host = max(dev.t_host, self_.t)
        return Ev()


def test_performance_ema_measures_device_time_not_enqueue_rate():
    """The reference's metric (tracker.performance_ema, callback.py:63): with a GPU stream that takes 10 ms
    per step while the host enqueues a step every 1 ms, the EMA must report the device's 100 steps/s
    (host perf_counter deltas would report ~1000)."""
    from dalle_amd.parallel.progress import PerformanceEMA

    fake = _FakeDevice(dev_ms=10.0)
    ema = PerformanceEMA(alpha=0.1, warmup=2)
    ema._events = True
    ema._record = fake.record
    for _ in range(60):
        fake.t_host += 1.0  # the host runs ahead
        ema.update(task_size=4)
    ema.flush()
    assert abs(ema.samples_per_second - 4 / 0.010) / (4 / 0.010) < 0.01, ema.samples_per_second
    assert ema.num_updates == 59 - 2  # 59 intervals, the first 2 dropped as warm-up
