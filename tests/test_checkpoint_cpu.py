"""Checkpoint / state formats the reference reads and writes (SURVEY §4 tier 7, §5.4): model_state.pt
(ModelWrapper keys, aliased shared-module keys, inference rename), state.zip backups and the
collaborative optimizer state_dict (8-bit LAMB states + local_epoch)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _task(tmp_path, **trainer_kw):
    from arguments import CollaborativeArguments, HFTrainerArguments, TrainingPeerArguments
    from task import TrainingTask

    peer = TrainingPeerArguments(authorize=False, experiment_prefix="ckpt", host_maddrs=["/ip4/127.0.0.1/tcp/0"],
                                 state_path=str(tmp_path / "state.zip"))
    tr = HFTrainerArguments(model_preset="tiny", text_seq_length=64, output_dir=str(tmp_path / "out"), **trainer_kw)
    collab = CollaborativeArguments(target_batch_size=4)
    return TrainingTask(peer, tr, collab), peer


def test_model_state_keys_aliases_and_resume(tmp_path):
    task, _ = _task(tmp_path)
    sd = task.model.state_dict()
    assert all(k.startswith("model.") for k in sd)
    # reversible layout + shared modules appear under every layer that uses them
    cfg = task.config
    qkv = [k for k in sd if k.endswith("to_qkv.weight")]
    assert len(qkv) == cfg.depth and all(".layers.blocks." in k and ".f.net." in k for k in qkv)
    assert "model.to_logits.1.weight" in sd and not any("text_emb.weight" in k for k in sd)
    ck = tmp_path / "out" / "checkpoint-7"
    ck.mkdir(parents=True)
    with torch.no_grad():
        for p in task.model.parameters():
            p.add_(0.5)
    torch.save(task.model.state_dict(), ck / "model_state.pt")
    task2, _ = _task(tmp_path)  # picks the newest checkpoint* dir up at init (task.py:88-93)
    for (n, a), (_, b) in zip(task.model.state_dict().items(), task2.model.state_dict().items()):
        assert torch.equal(a, b), n


def test_inference_rename_roundtrip(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "inference"))
    from run_inference import normalize_state_dict_keys

    task, _ = _task(tmp_path)
    sd = task.model.state_dict()
    # the reference's inference build inserts CachedAs levels: net.fn.fn -> net.fn.fn.fn, to_qkv -> fn.to_qkv
    renamed = {k.replace("net.fn.fn", "net.fn.fn.fn").replace("to_qkv", "fn.to_qkv").replace("to_out", "fn.to_out"): v
               for k, v in sd.items()}
    back = normalize_state_dict_keys(renamed)
    assert list(back.keys()) == list(sd.keys())
    assert normalize_state_dict_keys(sd).keys() == sd.keys()  # training-layout keys pass unchanged
    task.model.load_state_dict(back, strict=True)


def test_state_zip_and_optimizer_state(tmp_path):
    from callback import CollaborativeCallback

    task, peer = _task(tmp_path)
    opt = task.collaborative_optimizer
    model = task.model
    # one real local step so the 8-bit states exist
    batch = {"input_ids": torch.randint(2, 900, (2, 64)), "attention_mask": torch.ones(2, 64, dtype=torch.long),
             "image": torch.randint(0, 512, (2, 256))}
    model(**batch)["loss"].backward()
    opt.step(batch_size=4)  # reaches target_batch_size=4 -> global step
    assert opt.local_epoch == 1
    sd = opt.state_dict()
    assert sd["state"]["local_epoch"] == 1 and "param_groups" in sd
    big = [s for s in sd["state"].values() if isinstance(s, dict) and "state1" in s and s["state1"].numel() > 4096]
    assert big and all(s["state1"].dtype == torch.uint8 and {"qmap1", "qmap2", "absmax1", "absmax2", "step"} <= set(s)
                       for s in big)
    cb = CollaborativeCallback(task, peer)
    cb.backup_state()
    state = torch.load(peer.state_path, weights_only=True)
    assert set(state) == {"model", "training", "scheduler", "local_epoch"}
    before = {n: p.detach().clone() for n, p in model.named_parameters()}
    with torch.no_grad():
        for p in model.parameters():
            p.fill_(float("nan"))
    cb.restore_from_backup(peer.state_path)
    for n, p in model.named_parameters():
        assert torch.equal(p, before[n]), n
    assert opt.local_epoch == 1


def test_mis_keyed_checkpoints_are_rejected(tmp_path):
    """Both loaders are strict (reference inference/run_inference.py:119): a checkpoint with a renamed
    key must raise instead of silently keeping the current weights for that key -- the inference loader
    (with its explicit allow-list of recomputed buffers) and the backup restore (whose optimizer state
    would otherwise be loaded next to stale weights)."""
    import pytest

    from callback import CollaborativeCallback
    from dalle_amd.utils.checkpoint import load_state_dict_checked

    task, peer = _task(tmp_path)
    sd = task.model.state_dict()
    # the full key set loads; a derived buffer may be absent (it is recomputed from the config)
    assert load_state_dict_checked(task.model, sd) == []
    no_buf = {k: v for k, v in sd.items() if not k.endswith("pos_emb")}
    assert all(k.endswith("pos_emb") for k in load_state_dict_checked(task.model, no_buf))
    bad = dict(sd)
    key = next(k for k in bad if k.endswith("to_qkv.weight"))
    bad[key.replace("to_qkv", "to_qkv_renamed")] = bad.pop(key)
    with pytest.raises(RuntimeError, match="does not match"):
        load_state_dict_checked(task.model, bad)

    cb = CollaborativeCallback(task, peer)
    cb.backup_state()
    snap = torch.load(peer.state_path, weights_only=True)
    snap["model"] = bad
    torch.save(snap, peer.state_path)
    with pytest.raises(RuntimeError):
        cb.restore_from_backup(peer.state_path)
