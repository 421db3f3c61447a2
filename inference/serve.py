#!/usr/bin/env python3
"""Text -> image serving on MI355X: an HTTP front-end over the hipGraph decode engine, on one GPU or on
every GPU of a node (``--devices all``: one model copy, decode-engine cache and worker thread per GPU;
each request goes to the device with the fewest images queued).

The reference only has the offline batch script (``inference/run_inference.py``); this is its online
counterpart for deployment. Requests are queued and a single GPU worker thread forms batches:

* requests with the same sampling parameters (temperature, top-k, top-p) share a batch; the worker
  waits at most ``--batch-window-ms`` for more work after the first request, up to ``--max-batch``
  images (the decode engine's skinny-GEMM path covers batches <= 64);
* the batch is padded to the next power of two and run through a decode engine (two concurrent
  :class:`DecodeEngine` chains from batch 32 on) cached per
  padded size, so every shape's hipGraph is captured once and replayed for every later batch;
* codes are decoded by the VQGAN and returned as base64 PNGs together with per-request timings.

Endpoints: ``POST /generate`` ``{"prompts": [...], "images_per_prompt": 1, "temperature": 1.0,
"top_k": 256, "top_p": 1.0}``, ``GET /health``, ``GET /stats``. ``create_app`` builds the app around
an already-loaded model (tests, embedding into another service); ``main`` loads weights like
``run_inference.py`` and starts uvicorn.
"""
from __future__ import annotations

import argparse
import base64
import copy
import io
import os
import queue
import sys
import threading
import time
from concurrent.futures import Future
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dalle_amd.models.generation import DecodeEngine, make_decode_engine  # noqa: E402
from dalle_amd.utils.logging import get_logger  # noqa: E402

logger = get_logger(__name__)


def _png_b64(img: np.ndarray) -> str:
    from PIL import Image

    buf = io.BytesIO()
    Image.fromarray((np.clip(img, 0.0, 1.0) * 255.0 + 0.5).astype(np.uint8)).save(buf, format="PNG")
    return base64.b64encode(buf.getvalue()).decode("ascii")


class _Job:
    def __init__(self, prompts: List[str], n: int, key: Tuple[float, int, float]):
        self.prompts, self.n, self.key = prompts, n, key
        self.future: Future = Future()
        self.t_submit = time.perf_counter()

    @property
    def images(self) -> int:
        return len(self.prompts) * self.n


class BatchingGenerator:
    """Owns the model on one device; ``submit`` is thread-safe, all GPU work happens in one thread."""

    def __init__(self, model, tokenizer, device, max_batch: int = 64, batch_window_ms: float = 20.0):
        self.model, self.tokenizer, self.device = model, tokenizer, torch.device(device)
        self.max_batch = max(1, int(max_batch))
        self.window = batch_window_ms / 1000.0
        self.q: "queue.Queue[Optional[_Job]]" = queue.Queue()
        self.engines: Dict[int, DecodeEngine] = {}
        self.stats = {"requests": 0, "images": 0, "batches": 0, "gpu_seconds": 0.0}
        self._held: List[_Job] = []  # popped while batching but with other sampling parameters
        self._thread = threading.Thread(target=self._loop, name="dalle-serve-worker", daemon=True)
        self._thread.start()

    # -- API ------------------------------------------------------------------------------------
    def submit(self, prompts: List[str], images_per_prompt: int = 1, temperature: float = 1.0, top_k: int = 0,
               top_p: float = 1.0) -> Future:
        job = _Job(list(prompts), int(images_per_prompt), (float(temperature), int(top_k), float(top_p)))
        if not job.prompts or job.n < 1:
            raise ValueError("need at least one prompt and images_per_prompt >= 1")
        if job.images > self.max_batch:
            raise ValueError(f"a request may ask for at most {self.max_batch} images")
        self.q.put(job)
        return job.future

    def close(self):
        self.q.put(None)
        self._thread.join(timeout=60)

    # -- worker ---------------------------------------------------------------------------------
    def _next(self, timeout: Optional[float], held: bool = True) -> Optional[_Job]:
        if held and self._held:
            return self._held.pop(0)
        try:
            return self.q.get(timeout=timeout) if timeout is None or timeout > 0 else self.q.get_nowait()
        except queue.Empty:
            return None

    def _loop(self):
        torch.set_grad_enabled(False)
        if self.device.type == "cuda":
            # this thread's current device = the generator's: streams, hipGraph captures and the native
            # ops' stream lookups must bind to that GPU, not to GPU 0
            torch.cuda.set_device(self.device)
            # and a (non-blocking) stream of the worker's own: work on the legacy default stream would have to
            # synchronise with every blocking stream -- including a hipGraph capture running in another
            # generator's thread on the same GPU, which then fails ("legacy stream depend on a capturing stream")
            with torch.cuda.stream(torch.cuda.Stream(device=self.device)):
                self._serve()
        else:
            self._serve()

    def _serve(self):
        while True:
            first = self._next(None)
            if first is None:
                return
            batch, size = [first], first.images
            deadline = time.perf_counter() + self.window
            # same-parameter jobs set aside earlier join first, then new arrivals until the window closes
            later = [j for j in self._held if j.key != first.key]
            for j in [j for j in self._held if j.key == first.key]:
                if size + j.images <= self.max_batch:
                    batch.append(j)
                    size += j.images
                else:
                    later.append(j)
            self._held = later
            while size < self.max_batch:
                job = self._next(deadline - time.perf_counter(), held=False)
                if job is None:
                    break
                if job.key == first.key and size + job.images <= self.max_batch:
                    batch.append(job)
                    size += job.images
                else:
                    self._held.append(job)
                    if job.key == first.key:  # no room: it opens the next batch
                        break
            try:
                self._run(batch)
            except Exception as e:  # noqa: BLE001 - report to the callers, keep serving
                logger.exception("generation failed")
                for job in batch:
                    if not job.future.done():
                        job.future.set_exception(e)

    def _ids(self, prompts: List[str]) -> torch.Tensor:
        L = self.model.text_seq_len
        out = torch.full((len(prompts), L), 1, dtype=torch.long)  # pad = eos = 1 (task.py:59)
        for i, p in enumerate(prompts):
            ids = self.tokenizer(p, add_special_tokens=False, max_length=L, truncation=True)["input_ids"][:L]
            if ids:
                out[i, : len(ids)] = torch.tensor(ids, dtype=torch.long)
        return out

    def _run(self, batch: List[_Job]):
        prompts = [p for job in batch for p in job.prompts for _ in range(job.n)]
        n = len(prompts)
        padded = 1
        while padded < n:
            padded *= 2
        padded = min(padded, self.max_batch) if n <= self.max_batch else n
        ids = self._ids(prompts + [prompts[-1]] * (padded - n)).to(self.device)
        eng = self.engines.get(padded)
        if eng is None:
            eng = self.engines[padded] = make_decode_engine(self.model, padded, device=self.device)
        temperature, top_k, top_p = batch[0].key
        t0 = time.perf_counter()
        codes = eng.generate(self.model.prepare_text(ids), temperature=temperature, top_k=top_k, top_p=top_p)[:n]
        imgs = self.model.vae.decode(codes) if self.model.vae is not None else None
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        gpu_s = time.perf_counter() - t0
        arr = imgs.permute(0, 2, 3, 1).float().cpu().numpy() if imgs is not None else None
        self.stats["batches"] += 1
        self.stats["gpu_seconds"] += gpu_s
        off = 0
        for job in batch:
            k = job.images
            res = {"images": [_png_b64(a) for a in arr[off:off + k]] if arr is not None else [],
                   "codes": codes[off:off + k].cpu().tolist() if arr is None else None,
                   "batch_images": n, "batch_padded": padded, "generate_seconds": round(gpu_s, 4),
                   "queue_seconds": round(t0 - job.t_submit, 4)}
            off += k
            self.stats["requests"] += 1
            self.stats["images"] += k
            job.future.set_result(res)


class MultiDeviceGenerator:
    """One :class:`BatchingGenerator` per device (its own model copy, decode-engine cache and worker
    thread); ``submit`` routes each request to the device with the fewest images in flight, so a node's
    GPUs batch and decode independently. Same interface as a single generator."""

    def __init__(self, model, tokenizer, devices: List[str], max_batch: int = 64, batch_window_ms: float = 20.0):
        if not devices:
            raise ValueError("need at least one device")
        self.gens: List[BatchingGenerator] = []
        for i, d in enumerate(devices):
            m = model if i == len(devices) - 1 else copy.deepcopy(model)  # the last device takes the original
            self.gens.append(BatchingGenerator(m.to(d).eval(), tokenizer, d, max_batch, batch_window_ms))
        self.max_batch = self.gens[0].max_batch
        self._inflight = [0] * len(self.gens)
        self._lock = threading.Lock()

    @property
    def device(self) -> str:
        return ",".join(str(g.device) for g in self.gens)

    @property
    def engines(self) -> Dict[int, DecodeEngine]:
        out: Dict[int, DecodeEngine] = {}
        for g in self.gens:
            out.update(g.engines)
        return out

    @property
    def stats(self) -> Dict[str, float]:
        tot = {"requests": 0, "images": 0, "batches": 0, "gpu_seconds": 0.0}
        for g in self.gens:
            for k in tot:
                tot[k] += g.stats[k]
        tot["per_device_images"] = [g.stats["images"] for g in self.gens]
        return tot

    def submit(self, prompts: List[str], images_per_prompt: int = 1, temperature: float = 1.0, top_k: int = 0,
               top_p: float = 1.0) -> Future:
        n = len(prompts) * int(images_per_prompt)
        with self._lock:
            i = min(range(len(self.gens)), key=lambda k: (self._inflight[k], k))
            self._inflight[i] += n
        try:
            fut = self.gens[i].submit(prompts, images_per_prompt, temperature, top_k, top_p)
        except Exception:
            with self._lock:
                self._inflight[i] -= n
            raise

        def done(_f, i=i, n=n):
            with self._lock:
                self._inflight[i] -= n

        fut.add_done_callback(done)
        return fut

    def close(self):
        for g in self.gens:
            g.close()


def parse_devices(spec: str) -> List[str]:
    """``all`` -> every visible GPU; ``0,2`` -> those GPUs; ``cpu`` -> CPU (tests); default: one device."""
    if spec in (None, "", "auto"):
        return ["cuda:0" if torch.cuda.is_available() else "cpu"]
    if spec == "all":
        n = torch.cuda.device_count()
        return [f"cuda:{i}" for i in range(n)] if n else ["cpu"]
    return [d if (d.startswith("cuda") or d == "cpu") else f"cuda:{int(d)}" for d in spec.split(",")]


try:  # the HTTP layer is optional: BatchingGenerator works without fastapi / pydantic
    from pydantic import BaseModel, Field

    class GenerateRequest(BaseModel):
        prompts: List[str]
        images_per_prompt: int = Field(1, ge=1)
        temperature: float = Field(1.0, ge=0.0)
        top_k: int = Field(0, ge=0)
        top_p: float = Field(1.0, gt=0.0, le=1.0)
except ImportError:  # pragma: no cover
    GenerateRequest = None


def create_app(gen):
    """HTTP app around a :class:`BatchingGenerator` or :class:`MultiDeviceGenerator`."""
    from fastapi import FastAPI, HTTPException

    app = FastAPI(title="dalle-mi355x")

    @app.get("/health")
    def health():
        return {"ok": True, "device": str(gen.device), "max_batch": gen.max_batch}

    @app.get("/stats")
    def stats():
        s = dict(gen.stats)
        s["images_per_gpu_second"] = round(s["images"] / s["gpu_seconds"], 3) if s["gpu_seconds"] else None
        s["cached_batch_shapes"] = sorted(gen.engines)
        return s

    @app.post("/generate")
    def generate(req: GenerateRequest):
        try:
            fut = gen.submit(req.prompts, req.images_per_prompt, req.temperature, req.top_k, req.top_p)
        except ValueError as e:
            raise HTTPException(status_code=400, detail=str(e))
        return fut.result()

    return app


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default=None, help="DALL-E checkpoint (*.pt); random-init without")
    ap.add_argument("--model-preset", default="reference")
    ap.add_argument("--vqgan", default=None)
    ap.add_argument("--vqgan-config", default=None)
    ap.add_argument("--tokenizer", default="t5-small")
    ap.add_argument("--max-batch", type=int, default=64)
    ap.add_argument("--devices", default="auto", help='"all" GPUs of the node, a list like "0,1,2,3", or "auto" (one)')
    ap.add_argument("--batch-window-ms", type=float, default=20.0)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    args = ap.parse_args(argv)
    from run_inference import make_model, normalize_state_dict_keys
    from dalle_amd.models.vqgan import VQGanVAE

    torch.set_grad_enabled(False)
    devices = parse_devices(args.devices)
    tokenizer, wrapper = make_model(args.model_preset, args.tokenizer)
    if args.model:
        wrapper.load_state_dict(normalize_state_dict_keys(torch.load(args.model, map_location="cpu", weights_only=True)),
                                strict=False)
    wrapper.model.vae = VQGanVAE(args.vqgan, args.vqgan_config).eval()
    if len(devices) == 1:
        gen = BatchingGenerator(wrapper.model.to(devices[0]).eval(), tokenizer, devices[0], args.max_batch,
                                args.batch_window_ms)
    else:
        gen = MultiDeviceGenerator(wrapper.model.eval(), tokenizer, devices, args.max_batch, args.batch_window_ms)
    logger.info(f"serving on {gen.device}")
    import uvicorn

    uvicorn.run(create_app(gen), host=args.host, port=args.port)


if __name__ == "__main__":
    main()
