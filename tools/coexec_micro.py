"""Do two backward launches that only feed the optimizer overlap when they run together?
Times the DeepSet weight-gradient kernel (gine_deepset_bwd, slab left) and the dense-chain
weight-gradient engine (gine_chain_wgrad, slab left) at the cfg2 shape: each alone, back to
back on one stream, and on two streams at once (eager launches, HIP events).
    python tools/coexec_micro.py [--nodes 16000] [--reps 20]"""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "raincast-gnn_amd"))
import torch  # noqa: E402

from raincast_gnn import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=16000)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    N, M, F, H = a.nodes, 11, 35, 128
    P = _lib.ptr
    ens = torch.randn(N, M, F, device=dev)
    nb = ctypes.c_size_t(0)
    _lib.call("gine_deepset_mask_bytes", N, M, H, ctypes.byref(nb))
    mask = torch.randint(0, 255, (nb.value,), dtype=torch.uint8, device=dev)
    dr = torch.randn(N, H, device=dev)
    parts = ctypes.c_int32(0)
    _lib.call("gine_deepset_bwd_num_partials", N, H, ctypes.byref(parts))
    ds_slab = torch.empty(parts.value * (H * F + H), device=dev)
    t = {k: torch.randn(N, H, device=dev) for k in ("dh0", "r", "s", "u", "e", "de", "dt", "ds")}
    x = torch.randn(N, F, device=dev)
    fl = ctypes.c_size_t(0)
    _lib.call("gine_chain_bwd_slab_floats", N, H, F, ctypes.byref(fl))
    ch_slab = torch.empty(fl.value, device=dev)

    def ds_bwd(s):
        _lib.call("gine_deepset_bwd", P(ens), P(mask), P(dr), P(ds_slab), None, None, N, M, F,
                  H, s.cuda_stream)

    def ch_wgrad(s):
        _lib.call("gine_chain_wgrad", P(t["dh0"]), P(x), P(t["r"]), P(t["s"]), P(t["u"]),
                  P(t["e"]), P(t["de"]), P(t["dt"]), P(t["ds"]), P(ch_slab), None, None, 11.0,
                  None, None, None, None, None, None, N, H, F, s.cuda_stream)

    s0 = torch.cuda.current_stream(dev)
    s1 = torch.cuda.Stream(dev)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s0)
        for _ in range(a.reps):
            fn()
        s0.wait_stream(s1)
        e1.record(s0)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.reps

    def both_streams():
        s1.wait_stream(s0)
        ds_bwd(s0)
        ch_wgrad(s1)
        s0.wait_stream(s1)

    res = {"deepset_bwd": timed(lambda: ds_bwd(s0)), "chain_wgrad": timed(lambda: ch_wgrad(s0)),
           "sequential": timed(lambda: (ds_bwd(s0), ch_wgrad(s0))),
           "two_streams": timed(both_streams)}
    print({k: round(v, 2) for k, v in res.items()})


if __name__ == "__main__":
    main()
