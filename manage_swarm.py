#!/usr/bin/env python3
"""Single-node swarm manager (the MI355X counterpart of the reference's ``manage_scaleset.py``):
``python manage_swarm.py up --trainers 8 --gpus 0,1,2,3,4,5,6,7 -- --model_preset bench24 ...``.
See ``dalle_amd/utils/swarm.py``."""
import sys

from dalle_amd.utils.swarm import _cli

if __name__ == "__main__":
    sys.exit(_cli())
