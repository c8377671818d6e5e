"""Phase profile of the one-launch GINE layer forward (every workgroup's s_memtime stamps).
    GINE_HIP_LIB=.../var/layerprof/libgine_hip.so python tools/layer_prof.py [--config 2]
Stamps of thread 0 per workgroup (gine_mpmlp.hip GINE_LAYER_PROFILE): 0 entry -> 1 matrix
role done -> 2 phase A done (block) -> 3 barrier arrival -> 4 grid barrier passed -> 5
BatchNorm finish + W2 fragments -> 6 relu(bn(a1)) in LDS -> 7 last Linear2 chain done."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raincast-gnn_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from raincast_gnn import _lib  # noqa: E402
from raincast_gnn import functional as Fn  # noqa: E402
from raincast_gnn.graph import GineGraph  # noqa: E402
from helpers import knn_batch_graph  # noqa: E402

CONFIGS = {1: (500, 10, 1), 2: (500, 10, 32)}
TICK_NOTE = "s_memtime ticks (shader clock)"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-stamps", action="store_true", help="plain library: time only")
    ap.add_argument("--no-win", action="store_true", help="gather from L2 (no layer windows)")
    ap.add_argument("--head", type=int, default=None, metavar="KIND",
                    help="fold the output head (GINE_LOSS_* kind, with a valid-target count) "
                         "into the launch (gine_layer_head)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    D = 128
    n, k, B = CONFIGS[a.config]
    ei, ea, N = knn_batch_graph(n, k, B, seed=0)
    from raincast_gnn.data import relabel_edges, station_order
    ei = relabel_edges(ei, station_order(ei[:, :ei.size(1) // B], n))
    ei, ea = ei.to(dev), ea.to(dev)
    g = GineGraph(ei, ea, N)
    assert Fn.layer_forward_ok(N, D, g.max_in_degree), "no one-launch layer at this size"
    torch.manual_seed(0)
    x = torch.randn(N, D, device=dev)
    lw, lb = torch.randn(D, device=dev), torch.randn(D, device=dev)
    ep = torch.tensor([0.1], device=dev)
    w1, w2 = (torch.randn(D, D, device=dev) / D ** 0.5 for _ in range(2))
    b1, b2 = torch.randn(D, device=dev), torch.randn(D, device=dev)
    gam, bet = torch.ones(D, device=dev), torch.zeros(D, device=dev)
    rm, rv = torch.zeros(D, device=dev), torch.ones(D, device=dev)
    z, a1, y = (torch.empty_like(x) for _ in range(3))
    mask = torch.empty(N, D, dtype=torch.uint8, device=dev)
    bsave = torch.empty(4, D, device=dev)
    acc = torch.zeros(Fn._count64("gine_bn_acc_words", D), dtype=torch.int64, device=dev)
    call, ptr = _lib.call, _lib.ptr
    ptr_ = ptr
    s = _lib.stream_handle(dev)
    lin = Fn.edge_linear_flag()
    win_args = (None, 0) if a.no_win else Fn.layer_window_args(g)
    print(f"layer windows: {'off (L2 gather)' if win_args[0] is None else win_args[1:]}")
    hargs = None
    if a.head is not None:
        K = {0: 2, 1: 3, 2: 4, 3: 5}[a.head]
        hw, hb = torch.randn(K, D, device=dev) / D ** 0.5, torch.randn(K, device=dev)
        raw, pred = torch.empty(N, K, device=dev), torch.empty(N, K, device=dev)
        yt = torch.randn(N, device=dev)
        parts = torch.empty(_lib.COUNT_PARTS, dtype=torch.int32, device=dev)
        hargs = ctypes.byref(_lib.LayerHead(ptr_(hw), ptr_(hb), ptr_(raw), ptr_(pred), ptr_(yt),
                                            ptr_(parts), a.head))
        print(f"head folded in: kind {a.head} (K = {K}), valid-target count")

    def run():
        call("gine_mp_fwd_layer", ptr(x), ptr(g.in_rowptr), ptr(g.in_src), ptr(g.in_attr),
             ptr(lw), ptr(lb), ptr(ep), ptr(w1), ptr(b1), ptr(z), ptr(a1), ptr(acc), ptr(gam),
             ptr(bet), ptr(rm), ptr(rv), None, ptr(bsave), 0.1, 1e-5, 1, ptr(w2), ptr(b2),
             ptr(y), ptr(mask), N, D, g.max_in_degree, lin, 2, *win_args, hargs, s)

    lib = _lib.load()
    buf = (ctypes.c_longlong * (1024 * 24))()
    P = Fn._count("gine_mlp_num_partials", N, D)
    names = ["matrix role", "phase A sync", "to arrival", "grid barrier", "BN finish + W2",
             "relu pass", "Linear2 chains"]
    for rep in range(0 if a.no_stamps else a.reps):
        run()
        torch.cuda.synchronize()
        lib.gine_debug_layer_prof(buf)
        full = np.frombuffer(buf, dtype=np.int64).reshape(1024, 24).astype(np.float64)
        # the workgroups of this launch: realtime entry stamps (one clock for all XCDs)
        # within 1 ms of the latest (the grid can be below P; older rows hold older runs)
        live = (full[:, 16] > 0) & (full[:, 16] > full[:, 16].max() - 1e5)
        full = full[live]
        t = full[:, :8]
        rel = t - t[:, 0].min()
        ph = np.diff(t, axis=1)
        if rep < a.reps - 1:
            continue
        print(f"cfg{a.config}: N={N}, {len(full)} workgroups (P = {P}); {TICK_NOTE} (last of "
              f"{a.reps} runs)")
        print(f"  span entry->last end {rel[:, 7].max():.0f}; entry: median "
              f"{np.median(rel[:, 0]):.0f} max {rel[:, 0].max():.0f}")
        print(f"  barrier arrival (mark 3): median {np.median(rel[:, 3]):.0f} max "
              f"{rel[:, 3].max():.0f}; release (mark 4): min {rel[:, 4].min():.0f} max "
              f"{rel[:, 4].max():.0f}")
        for i, nm in enumerate(names):
            print(f"  {nm:15s} median {np.median(ph[:, i]):8.0f}  p90 "
                  f"{np.percentile(ph[:, i], 90):8.0f}  max {ph[:, i].max():8.0f}")
        rt = (full[:, 16:20] - full[:, 16].min()) * 10.0  # 100 MHz ticks -> ns
        print(f"  realtime (ns after the first entry): entry median {np.median(rt[:, 0]):.0f} "
              f"p90 {np.percentile(rt[:, 0], 90):.0f} max {rt[:, 0].max():.0f}; barrier arrival "
              f"median {np.median(rt[:, 1]):.0f} max {rt[:, 1].max():.0f}; release min "
              f"{rt[:, 2].min():.0f} max {rt[:, 2].max():.0f}; end median {np.median(rt[:, 3]):.0f}"
              f" max {rt[:, 3].max():.0f}")
        arr = rt[:, 1] - rt[:, 0]
        print(f"  entry -> arrival (ns): median {np.median(arr):.0f} p90 "
              f"{np.percentile(arr, 90):.0f} max {arr.max():.0f}; latest-arriving workgroup "
              f"entered at {rt[np.argmax(rt[:, 1]), 0]:.0f}")
        # phase A detail, relative to each workgroup's entry (mark 0); workgroups with two
        # tiles only for the tile-2 marks
        two = full[:, 11] > full[:, 0]
        print(f"  phase A detail (ticks after entry, median over workgroups; {int(two.sum())} "
              f"with two tiles):")
        marks = [(8, "W1 planes ready"), (14, "tile 1 gathered"), (20, "tile 1 z ready"),
                 (9, "tile 1 chain"), (10, "tile 1 epilogue"), (15, "tile 2 gathered"),
                 (21, "tile 2 z ready"), (11, "tile 2 chain"),
                 (12, "tile 2 epilogue"), (13, "stats in acc"), (1, "matrix role end")]
        if win_args[0] is not None:  # window form: tile k's window staged (after G_k)
            marks[1:1] = [(22, "tile 1 staged")]
            marks[6:6] = [(23, "tile 2 staged")]
        for i, nm in marks:
            sel = two if i in (11, 12, 15, 21, 23) else np.ones_like(two)
            d = full[sel, i] - full[sel, 0]
            print(f"    {nm:16s} median {np.median(d):8.0f}  p90 {np.percentile(d, 90):8.0f}")
    # a reference: HIP-event time of the launch
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        run()
    st.record()
    for _ in range(20):
        run()
    en.record()
    torch.cuda.synchronize()
    print(f"  launch time (HIP events, 20 back to back): {st.elapsed_time(en) / 20 * 1e3:.2f} us")


if __name__ == "__main__":
    main()
