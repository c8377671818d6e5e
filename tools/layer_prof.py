"""The one-launch node-MLP backward (gine_mlp_bwd_layer) at cfg2's size against the pair it
replaces (gine_mlp_bwd2_acc + gine_mlp_bwd1_bn): HIP-event times of each form standalone,
and, with the phase-stamp build, workgroup 0's timeline (s_memtime cycles).
    python tools/layer_prof.py [--nodes 16000] [--epi 2]
    GINE_HIP_LIB=raincast-gnn_amd/raincast_gnn/_native/var/rgprof/libgine_hip.so python tools/layer_prof.py --stamps
Stamps: 10 start, 11 W2 planes ready, 12 tile staged, 13 chain done, 14 epilogue done,
15 BatchNorm sums performed, 16 W1 planes ready, 17 past the grid barrier, 18 BatchNorm
finished, 19 dz chain done, 20 dz stored."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raincast-gnn_amd")]
import torch  # noqa: E402

from raincast_gnn import _lib  # noqa: E402
from raincast_gnn import functional as Fn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=16000)
    ap.add_argument("--epi", type=int, default=2)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--stamps", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    N, D = a.nodes, 128
    torch.manual_seed(0)
    dy, a1 = torch.randn(N, D, device=dev), torch.randn(N, D, device=dev)
    y = torch.randn(N, D, device=dev)
    mask = (torch.rand(N, D, device=dev) > 0.5).to(torch.uint8)
    w1, w2 = torch.randn(D, D, device=dev) / 11, torch.randn(D, D, device=dev) / 11
    gamma = torch.rand(D, device=dev) + 0.5
    bn_save = torch.stack([a1.mean(0), 1 / a1.std(0), gamma / a1.std(0),
                           -a1.mean(0) * gamma / a1.std(0)]).contiguous()
    dbn, dz, dbn2, dz2 = (torch.empty_like(dy) for _ in range(4))
    coef = torch.empty(3, D, device=dev)
    dg, db = torch.empty(D, device=dev), torch.empty(D, device=dev)
    words = Fn._count64("gine_bn_acc_words", D)
    acc = torch.zeros(words, dtype=torch.int64, device=dev)
    s = _lib.stream_handle(dev)
    c, p = _lib.call, _lib.ptr

    def layer():
        c("gine_mlp_bwd_layer", p(dy), p(y), p(mask), p(a1), p(bn_save), p(w2), p(w1), p(dbn),
          p(acc), p(gamma), p(dg), p(db), p(coef), p(dz), N, D, a.epi, s)

    def pair():
        c("gine_mlp_bwd2_acc", p(dy), p(y), p(mask), p(a1), p(bn_save), p(w2), p(dbn2), None,
          p(acc), N, D, a.epi, s)
        c("gine_mlp_bwd1_bn", p(dbn2), p(a1), p(bn_save), p(acc), p(gamma), p(dg), p(db),
          p(coef), p(w1), p(dz2), N, D, s)

    def timed(fn):
        for _ in range(5):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.reps

    if a.stamps:
        buf = (ctypes.c_longlong * 4096)()
        n = ctypes.c_int(0)
        layer()
        c("gine_debug_rg_prof", buf, ctypes.byref(n))   # drop the warm-up's stamps
        layer()
        c("gine_debug_rg_prof", buf, ctypes.byref(n))
        t0 = buf[1]
        prev = t0
        for i in range(n.value):
            tag, t = buf[2 * i], buf[2 * i + 1]
            print(f"stamp {tag:3d}  +{t - t0:8d} cycles  (step {t - prev:7d})")
            prev = t
        return
    tl, tp = timed(layer), timed(pair)
    torch.cuda.synchronize()
    print(f"N={N} epi={a.epi}: layer {tl:.2f} us, pair {tp:.2f} us; "
          f"dz equal {torch.equal(dz, dz2)}, dbn equal {torch.equal(dbn, dbn2)}")


if __name__ == "__main__":
    main()
