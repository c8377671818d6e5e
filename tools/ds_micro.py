"""Microbenchmark of the fused DeepSet phi kernels at several node counts (HIP events).
    python tools/ds_micro.py [--reps 50] [--nodes 4000,8000,16000,32000]"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "raincast-gnn_amd"))
import torch  # noqa: E402

from raincast_gnn import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--nodes", default="4000,8000,16000,32000")
    ap.add_argument("--M", type=int, default=11)
    ap.add_argument("--F", type=int, default=35)
    ap.add_argument("--H", type=int, default=128)
    ap.add_argument("--bwd", action="store_true", help="--prof: profile the backward")
    ap.add_argument("--prof", action="store_true",
                    help="phase profile of the forward (needs GINE_HIP_LIB = the dsprof build)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    out = {}
    for N in map(int, a.nodes.split(",")):
        ens = torch.randn(N, a.M, a.F, device=dev)
        w = torch.randn(a.H, a.F, device=dev) / a.F ** 0.5
        b = torch.randn(a.H, device=dev) * 0.1
        r = torch.empty(N, a.H, device=dev)
        dr = torch.randn(N, a.H, device=dev)
        nbytes = ctypes.c_size_t(0)
        _lib.call("gine_deepset_mask_bytes", N, a.M, a.H, ctypes.byref(nbytes))
        mask = torch.empty(nbytes.value, dtype=torch.uint8, device=dev)
        parts = ctypes.c_int32(0)
        _lib.call("gine_deepset_bwd_num_partials", N, a.H, ctypes.byref(parts))
        slab = torch.empty(parts.value * (a.H * a.F + a.H), device=dev)
        dw = torch.empty(a.H, a.F, device=dev)
        db = torch.empty(a.H, device=dev)
        s = _lib.stream_handle(dev)
        fwd = lambda: _lib.call("gine_deepset_fwd", _lib.ptr(ens), _lib.ptr(w), _lib.ptr(b),
                                _lib.ptr(r), _lib.ptr(mask), N, a.M, a.F, a.H, s)
        bwd = lambda: _lib.call("gine_deepset_bwd", _lib.ptr(ens), _lib.ptr(mask), _lib.ptr(dr),
                                _lib.ptr(slab), _lib.ptr(dw), _lib.ptr(db), N, a.M, a.F, a.H, s)
        if a.prof:
            lib = _lib.load()
            buf = (ctypes.c_longlong * 4096)()
            n = ctypes.c_int(0)
            fwd()
            lib.gine_debug_ds_prof(buf, ctypes.byref(n))   # reset
            (bwd if a.bwd else fwd)()
            lib.gine_debug_ds_prof(buf, ctypes.byref(n))
            ev = [(buf[2 * i], buf[2 * i + 1]) for i in range(n.value)]
            names = ({0: "top", 1: "loads issued", 2: "dh", 3: "mfma + tail fma",
                      4: "body end", 5: "lds store", 6: "barrier"} if a.bwd else
                     {0: "top", 1: "loads issued", 2: "mfma chain", 3: "epilogue",
                      4: "mask store", 5: "lds store", 6: "barrier"})
            acc, cnt = {}, {}
            for (t0, c0), (t1, c1) in zip(ev, ev[1:]):
                if t1 == 0:
                    continue
                acc[t1] = acc.get(t1, 0) + (c1 - c0)
                cnt[t1] = cnt.get(t1, 0) + 1
            tot = sum(acc[k] / cnt[k] for k in acc)
            print(N, "phase cycles/tile (s_memtime):",
                  {names[k]: round(acc[k] / cnt[k]) for k in sorted(acc)}, "total", round(tot),
                  flush=True)
            continue
        res = {}
        for name, fn in (("fwd", fwd), ("bwd", bwd)):
            for _ in range(3):
                fn()
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(a.reps):
                fn()
            en.record()
            torch.cuda.synchronize()
            us = st.elapsed_time(en) * 1e3 / a.reps
            flops = 2.0 * N * a.M * a.F * a.H
            res[name] = {"us": round(us, 2), "TFLOPps": round(flops / us / 1e6, 2)}
        out[N] = res
        print(N, json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
