"""Generate tests/golden/reference_heads.npz from the REFERENCE's own modules.

Run in the build container only (needs /root/reference; the GPU box does not have it):
    python tests/golden/make_reference_heads.py

Imports models/model_utils.py (PostProcess) and models/loss.py (NormalCRPS,
MixedNormalCRPS, MixedLoss) from /root/reference -- both import and run without
torch_geometric -- evaluates them on seeded inputs and stores inputs,
post-processed parameters, losses and d(loss)/d(raw head output) as plain arrays.
Nothing from the reference is copied; only these numbers are committed.
"""
import os
import sys

import numpy as np
import torch

REF = os.environ.get("RAINCAST_REFERENCE", "/root/reference")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_heads.npz")

CASES = [  # (name, loss, grad_u string as in params.json, out_channels)
    ("normal", "NormalCRPS", "False", 2),
    ("normal_mixed", "MixedNormalCRPS", "False", 3),
    ("mixed", "MixedLoss", "False", 4),
    ("mixed_u", "MixedLoss", "True", 5),
]


def main():
    sys.path.insert(0, REF)
    from models.loss import MixedLoss, MixedNormalCRPS, NormalCRPS  # noqa: E402
    from models.model_utils import PostProcess  # noqa: E402

    g = torch.Generator().manual_seed(1234)
    n = 257
    arrays = {}
    for name, loss, grad_u, out in CASES:
        raw = torch.randn(n, out, generator=g, dtype=torch.float32)
        raw[:, 0] = raw[:, 0] * 2.0 - 1.0                     # mu spread around log-space
        r = torch.rand(n, generator=g)
        y = torch.where(r < 0.5, torch.full((n,), float(np.log(0.01))),
                        torch.randn(n, generator=g) * 1.5 + 0.5).to(torch.float32)
        y[torch.rand(n, generator=g) < 0.05] = float("nan")
        if loss == "NormalCRPS":
            fn = NormalCRPS()
        elif loss == "MixedNormalCRPS":
            fn = MixedNormalCRPS()
        elif grad_u == "True":
            fn = MixedLoss(grad_u=True, xi=0.5)
        else:
            fn = MixedLoss(grad_u=False, u=1.71, xi=0.5)
        x = raw.clone().requires_grad_(True)
        pp = PostProcess(loss, grad_u)(x)
        val = fn.crps(pp, y)
        val.backward()
        arrays[f"{name}_raw"] = raw.numpy()
        arrays[f"{name}_y"] = y.numpy()
        arrays[f"{name}_pp"] = pp.detach().numpy()
        arrays[f"{name}_loss"] = np.array([val.item()], dtype=np.float64)
        arrays[f"{name}_loss_dtype"] = np.array([str(val.dtype)])
        arrays[f"{name}_grad"] = x.grad.numpy()
    np.savez_compressed(OUT, **arrays)
    print(f"wrote {OUT} ({os.path.getsize(OUT)} bytes)")


if __name__ == "__main__":
    main()
