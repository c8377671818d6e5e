"""A/B bit-compare of the D=128 row GEMMs across builds/switches (GINE_HIP_LIB=variant .so):
    python tools/rowgemm_ab.py OUT.pt [--nodes 16000]   (run twice, then --compare A.pt B.pt)
Runs gine_mlp_fwd2 (3 epilogues), gine_mlp_bwd2 (3 epilogues) and gine_mlp_bwd1 on fixed
seeded inputs and saves every output (and the BN partial rows)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "raincast-gnn_amd"))
import torch  # noqa: E402

from raincast_gnn import _lib, functional as Fn  # noqa: E402


def run(N):
    dev = torch.device("cuda:0")
    D = 128
    g = torch.Generator(device="cpu").manual_seed(7)
    r = lambda *s: torch.randn(*s, generator=g).to(dev)  # noqa: E731
    x, a1, dy, dbn = r(N, D), r(N, D), r(N, D), r(N, D)
    y = r(N, D)
    w2, w1, b2 = r(D, D) / 11, r(D, D) / 11, r(D)
    bn_save = torch.cat([r(1, D) * 0.1, r(1, D).abs() + 0.5, r(1, D), r(1, D)]).contiguous()
    coef = r(3, D)
    mask = (r(N, D) > 0).to(torch.uint8)
    P = Fn._count("gine_mlp_num_partials", N, D)
    s = _lib.stream_handle(dev)
    p = _lib.ptr
    out = {}
    for epi in (0, 1, 2):
        yo = torch.empty(N, D, device=dev)
        m = torch.zeros(N, D, dtype=torch.uint8, device=dev)
        _lib.call("gine_mlp_fwd2", p(a1), p(bn_save), p(w2), p(b2), p(x), p(yo), p(m), N, D,
                  epi, s)
        out[f"fwd2_{epi}"] = yo
        out[f"fwd2_{epi}_mask"] = m
        d = torch.empty(N, D, device=dev)
        part = torch.empty(P, 2, D, dtype=torch.float64, device=dev)
        _lib.call("gine_mlp_bwd2", p(dy), p(y), p(mask), p(a1), p(bn_save), p(w2), p(d),
                  p(part), N, D, epi, s)
        out[f"bwd2_{epi}"] = d
        out[f"bwd2_{epi}_part_total"] = part.sum(0)
    dz = torch.empty(N, D, device=dev)
    _lib.call("gine_mlp_bwd1", p(dbn), p(a1), p(bn_save), p(coef), p(w1), p(dz), N, D, s)
    out["bwd1"] = dz
    torch.cuda.synchronize()
    return {k: v.cpu() for k, v in out.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out", nargs="?")
    ap.add_argument("--nodes", type=int, default=16000)
    ap.add_argument("--compare", nargs=2)
    a = ap.parse_args()
    if a.compare:
        A, B = (torch.load(f, weights_only=True) for f in a.compare)
        bad = 0
        for k in A:
            if k.endswith("part_total"):
                rel = ((A[k] - B[k]).abs().max() / B[k].abs().max()).item()
                print(f"{k}: rel {rel:.2e}")
                bad += rel > 1e-12
            else:
                eq = torch.equal(A[k], B[k])
                print(f"{k}: {'identical' if eq else 'DIFFERENT'}")
                bad += not eq
        sys.exit(1 if bad else 0)
    torch.save(run(a.nodes), a.out)


if __name__ == "__main__":
    main()
