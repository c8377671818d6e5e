"""Microbenchmark of the CRPS pass alone (gine_crps_fwd, 256 nodes per workgroup) at several
node counts -- a flat time over N means the pass is bound by one node's dependent chain.
    python tools/crps_micro.py [--nodes 1000,4000,16000,64000] [--kind 2] [--reps 50] [--head]
--head: the training step's form (gine_crps_head_fwd_grad: 64 nodes per workgroup, the
unit-seed gradient and the output head's backward in the same pass, D = 128)."""
import argparse
import ctypes
import json
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "raincast-gnn_amd"))
import torch  # noqa: E402

from raincast_gnn import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", default="1000,4000,16000,64000")
    ap.add_argument("--kind", type=int, default=2)  # GINE_LOSS_MIXED
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--head", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    K = {0: 2, 1: 3, 2: 4, 3: 5}[a.kind]
    for N in map(int, a.nodes.split(",")):
        g = torch.Generator(device="cpu").manual_seed(0)
        pred = torch.randn(N, K, generator=g)
        pred[:, 1] = pred[:, 1].abs() + 0.5          # sigma
        pred[:, 2] = torch.rand(N, generator=g)      # p
        if K > 3:
            pred[:, 3] = pred[:, 3].abs() + 0.5      # sigma_u
        pred = pred.to(dev).contiguous()
        y = (torch.randn(N, generator=g) * 2).to(dev)
        dpred = torch.empty(N, K, dtype=torch.float64, device=dev)
        n_part = ctypes.c_int32(0)
        _lib.call("gine_crps_num_partials", N, ctypes.byref(n_part))
        partials = torch.empty(n_part.value, 2, dtype=torch.float64, device=dev)
        loss = torch.empty(1, dtype=torch.float64, device=dev)
        count = torch.empty(1, dtype=torch.float64, device=dev)
        ticket = torch.zeros(1, dtype=torch.int32, device=dev)
        s = _lib.stream_handle(dev)
        if a.head:
            D = 128
            h = torch.randn(N, D, device=dev)
            w = torch.randn(K, D, device=dev) / D ** 0.5
            raw = torch.randn(N, K, device=dev)
            dh = torch.empty(N, D, device=dev)
            fl = ctypes.c_size_t(0)
            _lib.call("gine_crps_head_slab_floats", N, D, a.kind, ctypes.byref(fl))
            slab = torch.empty(fl.value, device=dev)
            parts = torch.empty(64, dtype=torch.int32, device=dev)
            _lib.call("gine_count_valid", _lib.ptr(y), N, _lib.ptr(parts), s)
            gu = torch.empty(N, K, device=dev)
            run = lambda: _lib.call("gine_crps_head_fwd_grad", _lib.ptr(pred), _lib.ptr(y), N,
                                    a.kind, 1.71, 0.5, math.log(0.01), 5.0, _lib.ptr(dpred),
                                    _lib.ptr(partials), _lib.ptr(loss), _lib.ptr(count),
                                    _lib.ptr(ticket), _lib.ptr(parts), _lib.ptr(gu),
                                    _lib.ptr(raw), _lib.ptr(h), _lib.ptr(w), D, _lib.ptr(dh),
                                    _lib.ptr(slab), s)
        else:
            run = lambda: _lib.call("gine_crps_fwd", _lib.ptr(pred), _lib.ptr(y), N, a.kind,
                                    1.71, 0.5, math.log(0.01), 5.0, _lib.ptr(dpred),
                                    _lib.ptr(partials), _lib.ptr(loss), _lib.ptr(count),
                                    _lib.ptr(ticket), s)
        for _ in range(3):
            run()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(a.reps):
            run()
        en.record()
        torch.cuda.synchronize()
        print(N, json.dumps({"us": round(st.elapsed_time(en) * 1e3 / a.reps, 2),
                             "loss": loss.item()}), flush=True)


if __name__ == "__main__":
    main()
