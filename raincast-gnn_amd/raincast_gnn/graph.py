"""Device-resident graph structures for the GINE kernels.

PyG gathers ``x[edge_index[0]]`` and scatter-adds into ``edge_index[1]`` on every call.
The MI355X engine instead sorts the edges once per distinct ``edge_index`` into two stable
CSR structures (in-edges by destination for the forward, out-edges by source for the
backward; see ``gine_graph_build`` in include/gine_hip.h) and reuses them for every layer.

The reference builds one static graph per station set (utils/data.py:261-284, shared by all
samples at utils/data.py:300) and PyG collates batches into a block-diagonal union, so in a
training run the same ``edge_index`` tensor (or a handful of them) recurs every step.
"""
from __future__ import annotations

import ctypes
from collections import OrderedDict

import torch

from . import _lib, options

# Window-staged message passing (gine_graph_plan_windows / gine_mp_*_win): channel-slice
# widths tried, the LDS bytes a window slice may take, and the tile size in nodes.
WINDOW_SLICES = (32, 16, 8)
WINDOW_ROW_BYTES = 64 * 1024
# LDS a window workgroup may take (a smaller budget for three workgroups per CU spilled:
# r02_s40)
WINDOW_LDS_BUDGET = _lib.WINDOW_LDS_BYTES


# A window launch has tiles x slices workgroups; below this many the gather kernels (one
# workgroup per 8 nodes) fill the chip better (measured: cfg1, 4 tiles, is slower staged).
# (The D = 64 sweep point, 125 tiles x 2 slices of 32 channels, is above it.)
WINDOW_MIN_WORKGROUPS = 200
# A plan whose windows together stage more than this many times the node table loses to
# the gather kernels (measured r02_s11: cfg5's 10,000-station k=32 graph in locality order
# plans 16-channel windows staging 10.8x the table, 186 us vs 118 us gathered; cfg2 in the
# dataset order stages 4.0x and wins, 15.4 vs 18.1 us).
WINDOW_MAX_STAGED = 6.0


def window_settings() -> tuple[str, int]:
    """(mode, max nodes per tile).  options.MP_WINDOW: "auto" (default) stages the
    backward only -- measured faster than the gather kernel at cfg2, while the staged
    forward is not --, "all" stages both directions, "0" uses the gather kernels."""
    mode = str(options.MP_WINDOW).lower()
    if mode in ("0", "off", "false", "none"):
        mode = "off"
    elif mode in ("1", "all", "on"):
        mode = "all"
    elif mode != "auto":
        raise ValueError(f"options.MP_WINDOW={mode!r}: expected auto, all or 0")
    return mode, int(options.WINDOW_NODES)


def plan_windows(rowptr: torch.Tensor, nbr: torch.Tensor, num_nodes: int, device,
                 max_nodes: int, max_staged: float | None = WINDOW_MAX_STAGED,
                 slots: bool = False) -> dict:
    """slice channels -> (WindowPlan, device arrays) or None, from a host copy of one CSR.
    ``max_staged`` rejects plans staging more than that many times the node table (None:
    keep every plan, MP_WINDOW "all").  ``slots``: add the degree-balanced work order of
    the backward (gine_graph_plan_window_slots).
    Blocks on the device (a D2H copy): call outside graph capture."""
    plans = {}
    if num_nodes == 0:
        return plans
    rp = rowptr.cpu()
    nb = nbr.cpu()
    i32 = dict(dtype=torch.int32)
    for cs in WINDOW_SLICES:
        max_rows = WINDOW_ROW_BYTES // (cs * 4)
        max_edges = (WINDOW_LDS_BUDGET - max_rows * cs * 4 - (max_nodes + 1) * 4) // 8
        tb = torch.empty(num_nodes + 1, **i32)
        lo = torch.empty(num_nodes, **i32)
        rows = torch.empty(num_nodes, **i32)
        maxima = torch.zeros(3, **i32)
        nt = ctypes.c_int32(0)
        _lib.call("gine_graph_plan_windows", rp.data_ptr(), nb.data_ptr(), num_nodes, max_rows,
                  max_nodes, max_edges, tb.data_ptr(), lo.data_ptr(), rows.data_ptr(),
                  ctypes.byref(nt), maxima.data_ptr())
        T = int(nt.value)
        if T == 0 or (max_staged is not None and int(rows[:T].sum()) > max_staged * num_nodes):
            plans[cs] = None
            continue
        edge_begin = rp[tb[:T + 1].long()].to(torch.int32)  # rowptr at the tile starts
        arrays = (tb[:T + 1].to(device), lo[:T].to(device), rows[:T].to(device),
                  edge_begin.to(device))
        m = [int(v) for v in maxima]
        plan = _lib.WindowPlan(arrays[0].data_ptr(), arrays[1].data_ptr(), arrays[2].data_ptr(),
                               T, cs, m[0], m[1], max(m[2], 1))
        plan.edge_begin = arrays[3].data_ptr()
        if slots:
            slot = torch.empty(num_nodes, dtype=torch.int16)
            _lib.call("gine_graph_plan_window_slots", rp.data_ptr(), tb.data_ptr(), T,
                      slot.data_ptr())
            arrays = arrays + (slot.to(device),)
            plan.slot = arrays[4].data_ptr()
        plans[cs] = (plan, arrays)
    return plans


class GineGraph:
    """Stable CSR (by destination) + CSR (by source) of one edge list on one device."""

    __slots__ = ("num_nodes", "num_edges", "device", "in_rowptr", "in_src", "in_attr",
                 "out_rowptr", "out_dst", "out_attr", "_error", "_checked", "_windows",
                 "max_in_degree", "_ext_opts", "layer_windows")

    def __init__(self, edge_index: torch.Tensor, edge_attr: torch.Tensor | None,
                 num_nodes: int, flow: str = "source_to_target"):
        _lib.require_device(edge_index, "GineGraph")
        self._ext_opts = {}  # torch_ext's per-size option cache
        if edge_index.dim() != 2 or edge_index.size(0) != 2:
            raise ValueError(f"edge_index must have shape [2, E], got {tuple(edge_index.shape)}")
        if flow not in ("source_to_target", "target_to_source"):
            raise ValueError(f"unknown flow '{flow}'")
        E = edge_index.size(1)
        if edge_attr is not None and edge_attr.numel() != E:
            raise ValueError(
                f"edge_attr must hold one value per edge (edge_dim=1): got shape "
                f"{tuple(edge_attr.shape)} for {E} edges")
        # PyG target_to_source: i = edge_index[0], j = edge_index[1] (flipped here)
        ei, attr = _canonical(edge_index, edge_attr, flow)
        dev = ei.device
        self.num_nodes, self.num_edges, self.device = int(num_nodes), int(E), dev
        i32 = dict(dtype=torch.int32, device=dev)
        self.in_rowptr = torch.empty(self.num_nodes + 1, **i32)
        self.out_rowptr = torch.empty(self.num_nodes + 1, **i32)
        self.in_src = torch.empty(max(E, 1), **i32)
        self.out_dst = torch.empty(max(E, 1), **i32)
        f32 = dict(dtype=torch.float32, device=dev)
        self.in_attr = torch.empty(max(E, 1), **f32) if attr is not None else None
        self.out_attr = torch.empty(max(E, 1), **f32) if attr is not None else None
        self._error = torch.zeros(1, **i32)
        ws_bytes = _lib.ctypes.c_size_t(0)
        _lib.call("gine_graph_workspace_bytes", self.num_nodes, E, _lib.ctypes.byref(ws_bytes))
        ws = torch.empty(max(int(ws_bytes.value), 1), dtype=torch.uint8, device=dev)
        with torch.cuda.device(dev):
            _lib.call("gine_graph_build", _lib.ptr(ei), _lib.ptr(attr), self.num_nodes, E,
                      _lib.ptr(self.in_rowptr), _lib.ptr(self.in_src), _lib.ptr(self.in_attr),
                      _lib.ptr(self.out_rowptr), _lib.ptr(self.out_dst), _lib.ptr(self.out_attr),
                      _lib.ptr(self._error), _lib.ptr(ws), ws.numel(), _lib.stream_handle(dev))
        # ws / ei / attr are freed on return: they were allocated on the current stream, so
        # the caching allocator only hands them out again to work ordered after the sort.
        self._checked = False
        self._windows = None
        self.max_in_degree = None  # host copy; None when built inside a stream capture
        self.layer_windows = None  # (tile windows, max rows, max in-edges) or None
        if not torch.cuda.is_current_stream_capturing():
            self.check()
            self._plan_windows()
            self.max_in_degree = int(self.in_degree().max()) if self.num_nodes > 0 else 0
            self._plan_layer_windows()

    def _plan_layer_windows(self) -> None:
        """The one-launch layer forward's per-tile windows (gine_graph_plan_layer_windows),
        kept when they fit its LDS with this graph's in-degree (gine_mp_fwd_layer_windows_fit):
        one small launch and one 8-byte readback per graph.  layer_windows = (tile windows
        [T, 2], largest window, largest in-edges of a tile)."""
        if self.num_nodes <= 0 or self.in_attr is None:
            return
        tiles = (self.num_nodes + 31) // 32
        win = torch.empty(tiles, 2, dtype=torch.int32, device=self.device)
        maxima = torch.empty(2, dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            _lib.call("gine_graph_plan_layer_windows", _lib.ptr(self.in_rowptr),
                      _lib.ptr(self.in_src), self.num_nodes, _lib.ptr(win), _lib.ptr(maxima),
                      _lib.stream_handle(self.device))
        rows, edges = (int(v) for v in maxima.tolist())
        ok = _lib.ctypes.c_int32(0)
        _lib.call("gine_mp_fwd_layer_windows_fit", rows, self.max_in_degree,
                  _lib.ctypes.byref(ok))
        if ok.value:
            self.layer_windows = (win, rows, edges)

    def _plan_windows(self) -> None:
        mode, max_nodes = window_settings()
        self._windows = {"in": {}, "out": {}}
        if mode == "off" or self.in_attr is None:
            return
        # "all" forces the staged kernels wherever a plan exists (tests, experiments); "auto"
        # keeps only plans that stage a bounded multiple of the table
        staged = None if mode == "all" else WINDOW_MAX_STAGED
        if mode == "all":
            self._windows["in"] = plan_windows(self.in_rowptr, self.in_src, self.num_nodes,
                                               self.device, max_nodes, staged)
        self._windows["out"] = plan_windows(self.out_rowptr, self.out_dst, self.num_nodes,
                                            self.device, max_nodes, staged, slots=True)
        self._windows["min_wg"] = 0 if mode == "all" else WINDOW_MIN_WORKGROUPS

    def window_plan_entry(self, side: str, channels: int):
        """(plan, device arrays) of the widest-slice window plan usable at this channel count
        (``side`` "in" for the forward, "out" for the backward), or None -> gather kernels."""
        if self._windows is None:
            return None
        for cs, entry in self._windows[side].items():
            if entry is not None and channels % cs == 0 and channels // cs <= 8:
                plan = entry[0]
                if plan.num_tiles * (channels // cs) < self._windows.get("min_wg", 0):
                    return None
                return entry
        return None

    def window_plan(self, side: str, channels: int):
        """The plan of :meth:`window_plan_entry` (a ctypes struct whose device arrays this
        graph owns: callers keep the graph alive while a launch may still use it)."""
        entry = self.window_plan_entry(side, channels)
        return None if entry is None else entry[0]

    def check(self) -> None:
        """Raise IndexError (like torch.index_select) when an index was out of range."""
        if self._checked:
            return
        if int(self._error.item()) != 0:
            raise IndexError(
                f"edge_index contains a node index outside [0, {self.num_nodes}) "
                "(index out of range in self)")
        self._checked = True

    def in_degree(self) -> torch.Tensor:
        return (self.in_rowptr[1:] - self.in_rowptr[:-1])

    def out_degree(self) -> torch.Tensor:
        return (self.out_rowptr[1:] - self.out_rowptr[:-1])


def _canonical(edge_index, edge_attr, flow="source_to_target"):
    """(int64 [2, E] contiguous 16-byte-aligned edge list in source->target orientation,
    fp32 [E] attributes or None) -- the form the graph build and the content check read."""
    ei = edge_index.to(torch.int64)
    if flow == "target_to_source":
        ei = ei.flip(0)
    ei = ei.contiguous()
    if ei.data_ptr() % 16:
        ei = ei.clone()
    attr = None
    if edge_attr is not None:
        attr = edge_attr.reshape(-1).to(dtype=torch.float32).contiguous()
        if attr.data_ptr() % 16:
            attr = attr.clone()
    return ei, attr


class _HostFlag:
    """Pinned host int32 slots per device that gine_graph_same_edges writes through their
    device mapping: the answers of content checks reach the host without a copy operation."""

    def __init__(self, device, slots: int):
        self.host = torch.zeros(slots, dtype=torch.int32, pin_memory=True)
        dp = ctypes.c_void_p(0)
        _lib.call("gine_host_device_ptr", self.host.data_ptr(), ctypes.byref(dp))
        self.dev_ptr = dp.value


class _GraphCache:
    """Graphs by tensor identity, and by content.

    * Identity: a small LRU keyed on the identity + version of the input tensors.  Entries
      hold strong references to the keyed tensors, so a cached pointer can never be recycled
      by the allocator for a different edge list while the entry lives; an in-place
      modification bumps ``_version`` and misses.
    * Content: the reference's training loop copies every batch to the device
      (``batch.to(device)``, train.py:62), so each step brings a NEW edge_index tensor
      holding the same static station graph (block-diagonally collated, utils/data.py:300).
      On an identity miss, the graphs built for the same (N, E, flow) -- up to
      ``per_shape`` distinct edge lists of that size, e.g. two station sets or radius graphs
      used alternately -- are checked against the new edge list on the device
      (gine_graph_same_edges, one pass over both per candidate, all candidates in one go)
      and the first equal one is reused with its CSRs, window plans and degree bound -- no
      sort, no host copy of the CSRs, no planning.
      COST: a content check waits for the current stream (one event synchronisation) before
      it can read its answer, i.e. it drains every kernel queued on that stream first.  The
      drop-in training loop syncs every step anyway (train.py:71 ``loss.item()``); a loop
      that passes the SAME edge_index tensor each step never pays it (identity hit).  Inside
      a stream capture (no synchronisation allowed) a miss builds as before.
    """

    def __init__(self, capacity: int = 8, content_capacity: int = 4, per_shape: int = 4):
        self.capacity = capacity
        self.content_capacity = content_capacity
        self.per_shape = per_shape
        self._entries: OrderedDict = OrderedDict()
        # shape key -> [(graph, ei, attr), ...] most recently used first
        self._content: OrderedDict = OrderedDict()
        self._flags: dict = {}
        self.stats = {"identity_hits": 0, "content_hits": 0, "builds": 0}

    @staticmethod
    def _key(edge_index, edge_attr, num_nodes, flow):
        def tk(t):
            if t is None:
                return None
            return (t.data_ptr(), t._version, tuple(t.shape), tuple(t.stride()), t.dtype)
        return (tk(edge_index), tk(edge_attr), int(num_nodes), flow, edge_index.device)

    def _remember(self, key, graph, edge_index, edge_attr):
        self._entries[key] = (graph, edge_index, edge_attr)
        while len(self._entries) > self.capacity:
            self._entries.popitem(last=False)

    def _first_same(self, dev, ei, attr, cands) -> int:
        """Index of the first candidate (graph, ref_ei, ref_attr) whose edge list (and
        attributes) equal ``ei`` / ``attr``, or -1: one device check per candidate into its
        own flag slot, then ONE synchronisation of the current stream."""
        flag = self._flags.get(dev)
        if flag is None:
            with torch.cuda.device(dev):
                flag = self._flags[dev] = _HostFlag(dev, self.per_shape)
        flag.host.zero_()
        stream = torch.cuda.current_stream(dev)
        for i, (_, ref_ei, ref_attr) in enumerate(cands):
            _lib.call("gine_graph_same_edges", ref_ei.data_ptr(), ei.data_ptr(),
                      _lib.ptr(ref_attr), _lib.ptr(attr), ei.size(1), flag.dev_ptr + 4 * i,
                      stream.cuda_stream)
        done = torch.cuda.Event()
        done.record(stream)
        done.synchronize()
        for i in range(len(cands)):
            if int(flag.host[i]) == 0:
                return i
        return -1

    def get(self, edge_index, edge_attr, num_nodes, flow="source_to_target") -> GineGraph:
        key = self._key(edge_index, edge_attr, num_nodes, flow)
        hit = self._entries.get(key)
        if hit is not None:
            self._entries.move_to_end(key)
            graph = hit[0]
            if not graph._checked and not torch.cuda.is_current_stream_capturing():
                graph.check()
            self.stats["identity_hits"] += 1
            return graph
        capturing = torch.cuda.is_current_stream_capturing()
        ckey = (int(num_nodes), int(edge_index.size(-1)), flow, edge_index.device,
                edge_attr is None)
        cands = self._content.get(ckey) if not capturing and edge_index.is_cuda else None
        if cands:
            ei, attr = _canonical(edge_index, edge_attr, flow)
            usable = [c for c in cands if c[0]._checked]
            i = self._first_same(edge_index.device, ei, attr, usable) if usable else -1
            if i >= 0:
                c = usable[i]
                cands.remove(c)
                cands.insert(0, c)
                self._content.move_to_end(ckey)
                self._remember(key, c[0], edge_index, edge_attr)
                self.stats["content_hits"] += 1
                return c[0]
        graph = GineGraph(edge_index, edge_attr, num_nodes, flow)
        self.stats["builds"] += 1
        self._remember(key, graph, edge_index, edge_attr)
        if not capturing and edge_index.is_cuda:
            ei, attr = _canonical(edge_index, edge_attr, flow)
            # private copies: an in-place change of the caller's tensor must not change
            # what later content checks compare against
            lst = self._content.setdefault(ckey, [])
            lst.insert(0, (graph, ei.clone(), None if attr is None else attr.clone()))
            del lst[self.per_shape:]
            self._content.move_to_end(ckey)
            while len(self._content) > self.content_capacity:
                self._content.popitem(last=False)
        return graph

    def clear(self) -> None:
        self._entries.clear()
        self._content.clear()


graph_cache = _GraphCache()


def get_graph(edge_index, edge_attr, num_nodes, flow="source_to_target") -> GineGraph:
    return graph_cache.get(edge_index, edge_attr, num_nodes, flow)
