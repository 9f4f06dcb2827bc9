"""Convert the reference's shipped example checkpoints to .npz fixtures (build container only).

    python oracle/convert_checkpoints.py

data/example_model/checkpoints/27776.pt (holonomic) and data/example_model_unicycle/checkpoints/55554.pt
(unicycle) are loaded with torch.load(weights_only=True) (no unpickling of code) and written as plain
float32 arrays, one per state_dict key, to tests/golden/ckpt_<step>.npz. The fixtures are data only; the
checkpoint files themselves never travel.
"""
import os

import numpy as np
import torch

REF = "/root/reference/data"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")

for sub, step in (("example_model", 27776), ("example_model_unicycle", 55554)):
    sd = torch.load(os.path.join(REF, sub, "checkpoints", "%d.pt" % step), map_location="cpu", weights_only=True)
    if not isinstance(sd, dict):
        raise SystemExit("%s: not a state_dict" % sub)
    arrs = {k: v.detach().cpu().numpy() for k, v in sd.items()}
    np.savez_compressed(os.path.join(OUT, "ckpt_%d.npz" % step), **arrs)
    print(sub, step, len(arrs), "tensors", sum(a.size for a in arrs.values()), "values")
