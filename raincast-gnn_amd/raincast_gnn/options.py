"""Engine path selection.

Every value here is the measured-best default of the path it selects; the alternatives stay
reachable because the engine needs them elsewhere (a shape the default cannot take: eval
mode, graphs without a window plan, more than 16,384 nodes, in-degree above 32) and because
the parity tests compare the paths with each other (tests set these attributes with
``monkeypatch.setattr``).  Nothing reads the environment: the product path has no tuning
switches.

MP_FUSED     "1": gine_mp_fwd_mlp1 (gather + Linear1 + BN statistics in one launch) where it
             applies (functional.fused_forward_ok); "0": never; "all": lift its size limit.
MP_WINDOW    "auto": LDS-window message-passing backward where a plan exists and the launch
             fills the chip; "all": every plan, both directions; "0": gather kernels only.
WINDOW_NODES nodes per window tile.
ENGINE_IN_MP True: the node-MLP weight-gradient engine runs inside the window backward
             launch (gine_mp_bwd_win_mlp_wgrad); False: beside the dz GEMM.
BN_ACC       True: BatchNorm statistics through the fixed-point accumulator (no finish
             launch) in training mode; False: fp64 partials + finish launch.
BN_ACC_BWD   the same for the BatchNorm backward sums.
LAYER_FWD    True: where the fused forward and the accumulator apply and the grid fits the
             device at once, the whole layer forward in one launch (gine_mp_fwd_layer: the
             fused forward and the second GEMM separated by a grid barrier); False: the pair.
LAYER_WIN    True: the one-launch layer forward stages each tile's neighbour rows (its window,
             gine_graph_plan_layer_windows) in LDS where the graph's plan fits; False (the
             measured-best default): it gathers them from L2.  Same bits either way; at cfg2
             the window form runs 27.2 against 24.6 us per launch.
LAYER_BWD    True: where the backward accumulator applies and the grid fits the device at
             once, the node-MLP backward in one launch (gine_mlp_bwd_layer: the dbn GEMM and
             the dz GEMM separated by a grid barrier); False: the pair.
HEAD_FOLD    True: the output head's forward (GNN.aggr + PostProcess, and the loss's
             valid-target count) runs in the last GINE layer's one-launch forward
             (gine_layer_head) where that launch applies; False: its own launch.  Same bits.
"""
from __future__ import annotations

MP_FUSED = "1"
MP_WINDOW = "auto"
WINDOW_NODES = 128
ENGINE_IN_MP = True
BN_ACC = True
BN_ACC_BWD = True
LAYER_FWD = True
LAYER_WIN = False
LAYER_BWD = True
HEAD_FOLD = True
