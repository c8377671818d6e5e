"""Drop-in ``GINEConv`` for the MI355X engine.

Mirrors ``torch_geometric.nn.GINEConv`` as models/gnn.py uses it:

* import        models/gnn.py:5    ``from torch_geometric.nn import GINEConv``
* construction  models/gnn.py:28   ``GINEConv(nn=mlp, train_eps=True, edge_dim=1)``
* call          models/gnn.py:41,44 ``conv(x, edge_index, edge_attr)``

Same constructor arguments, attributes (``nn``, ``eps``, ``lin``, ``initial_eps``),
state_dict keys (``nn.*``, ``eps``, ``lin.weight``, ``lin.bias``), ``reset_parameters``
and error behaviour.  ``forward`` runs the message passing in HIP and, when ``nn`` is
``Sequential(Linear(D,D), BatchNorm1d(D), ReLU(), Linear(D,D))`` with D in {32,64,128,256},
the node MLP too; any other ``nn`` is applied to the HIP-aggregated features as a module.
"""
from __future__ import annotations

import torch
from torch import Tensor
from torch.nn import BatchNorm1d, Linear, Parameter, ReLU, Sequential

from . import _lib, gradbuf, torch_ext
from .functional import (EPI_NONE, EPI_RELU, EPI_RESIDUAL_RELU, BnConfig, GineLayer,
                         GineMessagePassing)
from .graph import get_graph

FUSED_CHANNELS = (32, 64, 128, 256)
# False: the Python autograd Function everywhere (the tests compare the two bindings)
USE_TORCH_EXT = True


def _reset(module) -> None:
    """PyG ``torch_geometric.nn.inits.reset``: reset_parameters on the module or its children."""
    if hasattr(module, "reset_parameters"):
        module.reset_parameters()
    elif hasattr(module, "children"):
        for child in module.children():
            _reset(child)


class GINEConv(torch.nn.Module):
    r"""Graph isomorphism operator with edge features (Hu et al., 2020):

    .. math::
        \mathbf{x}^{\prime}_i = h_{\mathbf{\Theta}} \left( (1 + \epsilon) \cdot
        \mathbf{x}_i + \sum_{j \in \mathcal{N}(i)} \mathrm{ReLU}
        ( \mathbf{x}_j + \mathbf{e}_{j,i} ) \right)

    with :math:`\mathbf{e}_{j,i} = \mathrm{lin}(a_{j,i})` when ``edge_dim`` is given.
    """

    def __init__(self, nn: torch.nn.Module, eps: float = 0.0, train_eps: bool = False,
                 edge_dim: int | None = None, **kwargs):
        super().__init__()
        aggr = kwargs.pop("aggr", "add")
        if aggr not in ("add", "sum"):
            raise NotImplementedError(f"GINEConv aggr='{aggr}' is not supported (sum only)")
        self.flow = kwargs.pop("flow", "source_to_target")
        if self.flow not in ("source_to_target", "target_to_source"):
            raise ValueError(f"Expected 'flow' to be either 'source_to_target' or "
                             f"'target_to_source' (got '{self.flow}')")
        kwargs.pop("node_dim", None)
        if kwargs:
            raise TypeError(f"unexpected keyword arguments {sorted(kwargs)}")
        self.nn = nn
        self.initial_eps = eps
        if train_eps:
            self.eps = Parameter(torch.empty(1))
        else:
            self.register_buffer("eps", torch.empty(1))
        if edge_dim is not None:
            inner = self.nn[0] if isinstance(self.nn, Sequential) else self.nn
            if hasattr(inner, "in_features"):
                in_channels = inner.in_features
            elif hasattr(inner, "in_channels"):
                in_channels = inner.in_channels
            else:
                raise ValueError("Could not infer input channels from `nn`.")
            self.lin = Linear(edge_dim, in_channels)
        else:
            self.lin = None
        self.reset_parameters()

    def reset_parameters(self) -> None:
        _reset(self.nn)
        self.eps.data.fill_(self.initial_eps)
        if self.lin is not None:
            self.lin.reset_parameters()

    # ---------------------------------------------------------------------------------
    def _fusable(self, x: Tensor) -> bool:
        nn = self._modules.get("nn")
        if not (isinstance(nn, Sequential) and len(nn) == 4):
            return False
        mods = tuple(nn._modules.values())
        l1, bn, act, l2 = mods
        D = x.size(1)
        # the module-type part is cached per (D, the child modules themselves -- held, not
        # their ids, so a replaced child can never match a stale entry): the drop-in path calls
        # this every layer and step (host time; profiles/r04_s03_dropin_prof_cpp.txt)
        cached = self.__dict__.get("_fuse_key")
        if cached is None or cached[0] != D or any(a is not b for a, b in zip(cached[1], mods)):
            self.__dict__["_fuse_ok"] = (
                type(l1) is Linear and type(bn) is BatchNorm1d and type(act) is ReLU
                and type(l2) is Linear and bn.num_features == D and D in FUSED_CHANNELS)
            self.__dict__["_fuse_key"] = (D, mods)
        if not self.__dict__["_fuse_ok"]:
            return False
        # attributes a cached child can change in place: re-checked on every call
        w1, w2 = l1.weight, l2.weight
        return (l1.bias is not None and l2.bias is not None
                and w1.shape == (D, D) and w2.shape == (D, D)
                and w1.dtype == torch.float32 and w2.dtype == torch.float32
                and w1.device == x.device and w2.device == x.device)

    def _check_inputs(self, x, edge_index, edge_attr, size):
        if isinstance(x, (tuple, list)):
            if len(x) == 2 and x[0] is x[1]:
                x = x[0]
            else:
                raise NotImplementedError("bipartite (x_src, x_dst) inputs are not supported")
        if not isinstance(x, Tensor) or x.dim() != 2:
            raise ValueError("x must be a [num_nodes, channels] tensor")
        _lib.require_device(x, "GINEConv")
        if x.dtype != torch.float32:
            raise TypeError(f"GINEConv runs in fp32 (got {x.dtype}); cast with x.float() as "
                            "ResGnn does (models/gnn.py:36)")
        if size is not None and (size[0] not in (None, x.size(0)) or size[1] not in (None, x.size(0))):
            raise NotImplementedError("size must match x (no bipartite propagation)")
        if self.lin is None:
            if edge_attr is not None and edge_attr.size(-1) != x.size(-1):
                raise ValueError("Node and edge feature dimensionalities do not match. "
                                 "Consider setting the 'edge_dim' attribute of 'GINEConv'")
            raise NotImplementedError("GINEConv without edge_dim (edge features of width D) "
                                      "is not implemented on the MI355X engine; use edge_dim=1")
        if self.lin.in_features != 1:
            raise NotImplementedError(f"edge_dim={self.lin.in_features}: only edge_dim=1 "
                                      "(the reference configuration) is implemented")
        if edge_attr is None:
            raise ValueError("GINEConv with edge_dim requires edge_attr")
        if (edge_attr.dim() == 2 and edge_attr.size(1) != 1) or edge_attr.dim() > 2:
            raise ValueError(f"edge_attr must be [E, 1] for edge_dim=1, got {tuple(edge_attr.shape)}")
        if edge_attr.requires_grad:
            raise NotImplementedError("gradients w.r.t. edge_attr are not implemented")
        if self.lin.in_features == 1 and self.lin.out_features != x.size(1):
            raise ValueError(f"lin projects to {self.lin.out_features} channels, x has {x.size(1)}")
        return x

    def _run(self, x, edge_index, edge_attr, size, epilogue, head=None):
        x = self._check_inputs(x, edge_index, edge_attr, size)
        edge_attr = edge_attr.float()
        graph = get_graph(edge_index, edge_attr, x.size(0), self.flow)
        if self._fusable(x):
            l1, bn, _, l2 = self.nn
            ext = torch_ext.get() if USE_TORCH_EXT else None
            if ext is not None and gradbuf.slice_of(l1.weight) is None:
                # the drop-in path (no flat gradient buffer: the non-deferred backward) from
                # the C++ autograd binding -- the same launches, far less host time
                return torch_ext.layer(ext, x, self, graph, epilogue)
            return GineLayer.apply(x, self.lin.weight, self.lin.bias, self.eps, l1.weight,
                                   l1.bias, bn.weight, bn.bias, l2.weight, l2.bias, graph,
                                   BnConfig(bn), epilogue, head)
        z = GineMessagePassing.apply(x, self.lin.weight, self.lin.bias, self.eps, graph)
        out = self.nn(z)
        if epilogue == EPI_RELU:
            out = torch.relu(out)
        elif epilogue == EPI_RESIDUAL_RELU:
            out = x + torch.relu(out)
        return out

    def forward(self, x, edge_index: Tensor, edge_attr: Tensor | None = None,
                size=None) -> Tensor:
        return self._run(x, edge_index, edge_attr, size, EPI_NONE)

    def forward_relu(self, x, edge_index, edge_attr=None, head=None):
        """relu(self(x, ...)) with the ReLU fused into the last GEMM (ResGnn layer 0).
        ``head``: a head.HeadPlan when the output head reads this result (the stack's last
        layer), run in the same launch where the one-launch layer forward applies."""
        return self._run(x, edge_index, edge_attr, None, EPI_RELU, head)

    def forward_residual_relu(self, x, edge_index, edge_attr=None, head=None):
        """x + relu(self(x, ...)) fused (ResGnn layers >= 1, models/gnn.py:44); ``head`` as
        for forward_relu."""
        return self._run(x, edge_index, edge_attr, None, EPI_RESIDUAL_RELU, head)

    def __repr__(self) -> str:
        return f"{self.__class__.__name__}(nn={self.nn})"
