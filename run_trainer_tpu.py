#!/usr/bin/env python3
"""Multi-device single-host trainer (counterpart of the reference ``run_trainer_tpu.py`` + ``lib/training/tpu.py``).

The reference drives 8 TPU cores from one host process (host master params + grads, per-core
replicas, explicit grad all-reduce into the host master, params pushed after each global step). On
a MI355X node the same pattern is one process per GPU with RCCL over xGMI: this entrypoint spawns
``--num_tpus`` local workers (one per GPU; CPU/gloo workers when no GPU is visible), each running the
collaborative training loop of ``run_trainer.py``. It also fixes the reference's stale pieces
(``n_tpus`` vs ``num_tpus``, the removed ``callbacks`` API).
"""
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    num = 8
    if "--num_tpus" in argv:
        i = argv.index("--num_tpus")
        num = int(argv[i + 1])
        del argv[i:i + 2]
    for flag in ("--wandb_project",):
        if flag in argv:
            i = argv.index(flag)
            del argv[i:i + 2]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(num),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "run_trainer.py"), *argv]
    return subprocess.call(cmd)


if __name__ == "__main__":
    sys.exit(main())
