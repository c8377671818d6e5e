"""Compare saved dx tensors of determinism_layer.py runs: rows and columns that differ."""
import sys
import torch
ref = torch.load(sys.argv[1], weights_only=True)["dx"]
for f in sys.argv[2:]:
    d = torch.load(f, weights_only=True)["dx"]
    bad = (d != ref)
    rows = bad.any(1).nonzero().flatten()
    cols = bad.any(0).nonzero().flatten()
    print(f, "rows differing", rows.numel(), "first", rows[:20].tolist(), "cols", cols.numel(),
          cols[:40].tolist(), "maxabs", (d - ref).abs().max().item(), "refmax", ref.abs().max().item())
    if rows.numel():
        r = rows[0].item()
        c = bad[r].nonzero().flatten()[:8].tolist()
        print("  row", r, "cols", c, "got", d[r, c].tolist(), "ref", ref[r, c].tolist())
