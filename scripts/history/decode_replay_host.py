#!/usr/bin/env python3
"""Is the captured decode step host-bound? Times the HOST side of graph.replay() (enqueue only) against the
device time of the same steps (reference model, batch 64, after the caption prefill)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.getcwd())
from dalle_amd.config import reference  # noqa: E402
from dalle_amd.models.dalle import DALLE  # noqa: E402
from dalle_amd.models.generation import make_decode_engine  # noqa: E402

dev = torch.device("cuda")
cfg = reference()
torch.manual_seed(0)
model = DALLE(cfg).to(dev).eval()
B = int(os.environ.get("B", "64"))
text = torch.randint(2, cfg.num_text_tokens, (B, cfg.text_seq_len), device=dev)
eng = make_decode_engine(model, B, device=dev)
model._decode_engine = eng
model.generate_images(text, top_k=256, use_graph=True, return_codes=True)
eng = model._decode_engine
torch.cuda.synchronize()
tb = model.prepare_text(text)
getattr(eng, "prefill_parallel", eng.prefill)(tb)
torch.cuda.synchronize()
graphs = [eng.graph] if getattr(eng, "graph", None) is not None else eng._graphs
K = 32
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
t0 = time.perf_counter()
for _ in range(K):
    for g in graphs:
        g.replay()
t_host = (time.perf_counter() - t0) / K
b.record()
torch.cuda.synchronize()
t_dev = a.elapsed_time(b) / K
print(json.dumps({"batch": B, "parts": getattr(eng, "nparts", 1), "graphs": len(graphs),
                  "host_ms_per_step_enqueue": round(t_host * 1e3, 3), "device_ms_per_step": round(t_dev, 3)}))
