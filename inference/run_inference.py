#!/usr/bin/env python3
"""Text -> image generation (reference ``inference/run_inference.py:1-146``), CLI-compatible.

For every query: 16 x 8 = 128 images (temperature / top-k / top-p sampling with the KV-cache decoder,
one hipGraph-captured step replayed per image token on MI355X), decoded by the VQGAN, optionally
re-ranked with the native CLIP ViT-B/32 (``dalle_amd.models.clip``; weights from ``--clip`` -- a
safetensors / state-dict file in OpenAI key layout -- or random-init with ``--clip random``; without
``--clip`` the scores are uniform), and saved as ``{output_dir}/{query}.pickle`` with keys
``query, temperature, images, clip_scores``.

Checkpoints in the training layout are accepted (the reference's CachedAs rename
``net.fn.fn -> net.fn.fn.fn`` / ``to_qkv -> fn.to_qkv`` / ``to_out -> fn.to_out`` is undone when present).
"""
import argparse
import copy
import os
import pickle
import sys
from collections import OrderedDict
from datetime import datetime

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dalle_amd.config import get_config  # noqa: E402
from dalle_amd.data.tokenizer import load_tokenizer  # noqa: E402
from dalle_amd.models.dalle import DALLE  # noqa: E402
from dalle_amd.models.vqgan import VQGanVAE  # noqa: E402



class ModelWrapper(torch.nn.Module):
    def __init__(self, model):
        super().__init__()
        self.model = model

    def forward(self, input_ids, attention_mask, image):
        return {'loss': self.model.forward(text=input_ids, image=image, mask=attention_mask, return_loss=True)}


def make_model(preset: str = "reference", tokenizer_path: str = "t5-small"):
    cfg = get_config(preset)
    tokenizer = load_tokenizer(tokenizer_path, vocab_size=cfg.num_text_tokens)
    tokenizer.pad_token = tokenizer.eos_token
    return tokenizer, ModelWrapper(DALLE(cfg))


def normalize_state_dict_keys(state_dict):
    """Map inference-layout (CachedAs) keys back onto the training layout; training-layout keys pass.

    The reference renames training keys for its inference model with
    ``net.fn.fn -> net.fn.fn.fn``, ``to_qkv -> fn.to_qkv``, ``to_out -> fn.to_out``
    (``inference/run_inference.py:117``): attention weights gain two ``fn`` levels
    (``f.net.fn.fn.fn.fn.fn.to_qkv``), feed-forward weights one (``g.net.fn.fn.fn.fn.net.0``).
    """
    out = OrderedDict()
    for k, v in state_dict.items():
        if ".fn.fn.fn.fn.fn.to_" in k:
            k = k.replace(".fn.fn.fn.fn.fn.to_", ".fn.fn.fn.to_")
        elif "net.fn.fn.fn.fn.net." in k:
            k = k.replace("net.fn.fn.fn.fn.net.", "net.fn.fn.fn.net.")
        out[k] = v
    return out


def generate(query, *, tokenizer, model, batch_size, n_iters, temperature, top_k, top_p, text_seq_len=256, device="cuda"):
    ids = tokenizer(query, add_special_tokens=False, max_length=text_seq_len, truncation=True)['input_ids']
    input_ids = torch.full((text_seq_len,), 1, dtype=torch.long)
    input_ids[: len(ids)] = torch.tensor(ids, dtype=torch.long)
    input_ids = input_ids.repeat(batch_size, 1).to(device)
    result = []
    for _ in range(n_iters):
        output = model.model.generate_images(input_ids, temperature=temperature, top_k=top_k, top_p=top_p, use_cache=True)
        output = output.permute(0, 2, 3, 1).float().cpu().numpy()
        result.extend(output)
    return result


def parse_devices(spec):
    """``all`` -> every visible GPU, ``0,2`` -> those GPUs, ``cpu`` (tests); default: one device."""
    if spec in (None, "", "auto"):
        return ["cuda" if torch.cuda.is_available() else "cpu"]
    if spec == "all":
        n = torch.cuda.device_count()
        return [f"cuda:{i}" for i in range(n)] if n else ["cpu"]
    return [d if (d.startswith("cuda") or d == "cpu") else f"cuda:{int(d)}" for d in spec.split(",")]


def run_queries(queries, per_device, work, device_of=None):
    """Spread ``queries`` over the devices: one worker thread per entry of ``per_device`` (its device's
    model copy and state), each taking the next unclaimed query -- GPUs finish at their own pace.
    ``device_of(ctx)`` names the entry's device: its thread makes it the CURRENT device, so streams,
    graph captures and the native ops' stream lookups bind to that GPU and not to GPU 0."""
    import queue
    import threading

    q = queue.Queue()
    for item in queries:
        q.put(item)
    errors = []

    def worker(ctx):
        dev = torch.device(device_of(ctx)) if device_of is not None else None
        if dev is not None and dev.type == "cuda":
            torch.cuda.set_device(dev)
        while not errors:
            try:
                item = q.get_nowait()
            except queue.Empty:
                return
            try:
                work(item, ctx)
            except BaseException as e:  # noqa: BLE001 - surfaced after the join
                errors.append(e)

    if len(per_device) == 1:
        worker(per_device[0])
    else:
        threads = [threading.Thread(target=worker, args=(ctx,), daemon=True) for ctx in per_device]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
    if errors:
        raise errors[0]


def load_queries(path: str):
    """One caption per line; trailing whitespace dropped, empty lines skipped (the reference's format)."""
    with open(path, encoding="utf-8") as fh:
        return [q for q in (raw.rstrip() for raw in fh) if q]


def main(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument('--queries', type=str, help='List of queries (*.txt, newline-separated)')
    parser.add_argument('--temperature', type=float, help='Sampling temperature', default=1.0)
    parser.add_argument('--top-k', type=int, default=0)
    parser.add_argument('--top-p', type=float, default=1.0)
    parser.add_argument('--model', type=str, help='DALL-E checkpoint (*.pt)', default=None)
    parser.add_argument('--vqgan', type=str, help='VQGAN checkpoint (*.ckpt)', default=None)
    parser.add_argument('--vqgan-config', type=str, help='VQGAN config (*.yaml)', default=None)
    parser.add_argument('--output-dir', type=str, help='Output directory')
    parser.add_argument('--model-preset', type=str, default='reference', help='[new] dalle_amd.config preset')
    parser.add_argument('--batch-size', type=int, default=16, help='[new] images per generate call (reference: 16)')
    parser.add_argument('--n-iters', type=int, default=8, help='[new] generate calls per query (reference: 8)')
    parser.add_argument('--clip', type=str, default=None, help='[new] CLIP ViT-B/32 weights (safetensors/state dict) or "random"')
    parser.add_argument('--clip-tokenizer', type=str, default=None, help='[new] CLIP BPE tokenizer.json (tokenizers format)')
    parser.add_argument('--devices', type=str, default='auto',
                        help='[new] "all" GPUs of the node or a list like "0,1": queries are spread over per-GPU workers')
    args = parser.parse_args(argv)
    torch.set_grad_enabled(False)  # inference only (the reference disabled grads at import time)

    queries = load_queries(args.queries)
    print(f'[*] Loaded {len(queries)} queries')

    devices = parse_devices(args.devices)
    tokenizer, model = make_model(args.model_preset)
    if args.model is not None:
        print(f'[*] Model modification time: {datetime.fromtimestamp(os.stat(args.model).st_mtime)}')
        state_dict = normalize_state_dict_keys(torch.load(args.model, map_location="cpu", weights_only=True))
        from dalle_amd.utils.checkpoint import load_state_dict_checked

        tolerated = load_state_dict_checked(model, state_dict)  # strict, as the reference (run_inference.py:119)
        print(f'[*] Loaded model' + (f' (recomputed buffers: {tolerated})' if tolerated else ''))
    else:
        print('[*] No --model given: random-init weights')

    gan = VQGanVAE(args.vqgan, args.vqgan_config)
    model.model.vae = gan.eval()
    # one model copy per device (the last device takes the original)
    models = [(model if i == len(devices) - 1 else copy.deepcopy(model)).to(d).eval() for i, d in enumerate(devices)]

    clip_models, clip_tok = [None] * len(devices), None
    if args.clip:
        from dalle_amd.models.clip import ClipTokenizer, load_clip

        clip_models = [load_clip(None if args.clip == "random" else args.clip, device=d) for d in devices]
        clip_tok = ClipTokenizer(args.clip_tokenizer)
        print(f"[*] CLIP ViT-B/32 {'random-init (scores are not meaningful)' if args.clip == 'random' else 'from ' + args.clip}")
    else:
        print('[*] No --clip weights: clip_scores will be uniform')

    os.makedirs(args.output_dir, exist_ok=True)
    print(f'[*] Saving results to `{args.output_dir}`')
    if len(devices) > 1:
        print(f'[*] {len(devices)} devices: {", ".join(devices)}')

    def work(query, ctx):
        model, clip_model, device = ctx
        images = generate(query, tokenizer=tokenizer, model=model, batch_size=args.batch_size, n_iters=args.n_iters,
                          temperature=args.temperature, top_k=args.top_k, top_p=args.top_p,
                          text_seq_len=model.model.text_seq_len, device=device)
        if clip_model is not None:
            from dalle_amd.models.clip import clip_scores as score_images

            clip_scores = score_images(clip_model, clip_tok, torch.from_numpy(np.stack(images)), query).cpu().numpy()
        else:
            clip_scores = np.full(len(images), 1.0 / len(images), dtype=np.float32)
        with open(os.path.join(args.output_dir, f'{query}.pickle'), 'wb') as f:
            outputs = {'query': query, 'temperature': args.temperature, 'images': images, 'clip_scores': clip_scores}
            pickle.dump(outputs, f)

    run_queries(queries, list(zip(models, clip_models, devices)), work, device_of=lambda ctx: ctx[2])


if __name__ == '__main__':
    main()
