import sys, torch
sys.path.insert(0, "/root/repo")
from dalle_amd.config import get_config
from dalle_amd.data.synthetic import synthetic_batch
from dalle_amd.models.dalle import DALLE
from dalle_amd.optim import FlatArena
from dalle_amd.ops import hip_ops
cfg = get_config("reference"); cfg.reversible_recompute = "auto"
dev = torch.device("cuda", 0)
m = DALLE(cfg).to(dev)
m.grad_arena = FlatArena(m.parameters(), device=dev)
b = synthetic_batch(4, cfg.text_seq_len, cfg.image_seq_len, cfg.num_text_tokens, cfg.num_image_tokens, device=dev)
hip_ops.PATH_COUNTS.clear()
loss = m(b["input_ids"], b["image"], mask=b["attention_mask"], return_loss=True); loss.backward(); torch.cuda.synchronize()
print("paths", dict(hip_ops.PATH_COUNTS))
