"""Inference / checkpoint-ensemble evaluation on the engine (eval.py:57-69, 153-218).

``predict_model`` runs the model in eval mode under ``no_grad`` over batches (BatchNorm from
its running statistics: the GINE layers' node MLP then takes the eval branch of
``gine_bn_fwd_finalize``) and concatenates the predictions; ``predict_ensemble`` averages
the predictions of several checkpoints (``stack(...).mean(0)``, eval.py:208-212) and
``ensemble_crps`` scores them with the model's own loss, as eval.py:216-218 does.
Checkpoints load with ``torch.load(weights_only=True)``: a state_dict is plain tensors.
"""
from __future__ import annotations

from typing import Iterable

import torch

from .data import restore_node_order


@torch.no_grad()
def predict_model(model: torch.nn.Module, batches: Iterable, device) -> torch.Tensor:
    """eval.py:57-69: eval mode, one forward per batch, predictions concatenated on the CPU
    (rows in the collated order of each batch, whatever order the batch is stored in)."""
    model.eval()
    # batches in the engine's station order come back in the reference (collated) order
    out = [restore_node_order(model(b.to(device)), b).cpu() for b in batches]
    return torch.cat(out, dim=0)


def predict_ensemble(make_model, checkpoints, batches, device) -> torch.Tensor:
    """eval.py:178-212: one model per checkpoint (state_dict path or dict), predictions
    averaged over checkpoints.  ``batches`` is re-iterated per checkpoint."""
    batches = list(batches)
    preds = []
    for ck in checkpoints:
        model = make_model().to(device)
        state = torch.load(ck, map_location=device, weights_only=True) if isinstance(ck, str) \
            else ck
        model.load_state_dict(state)
        preds.append(predict_model(model, batches, device))
    if len(preds) == 1:
        return preds[0]
    return torch.stack(preds, dim=0).mean(dim=0)


def ensemble_crps(model: torch.nn.Module, preds: torch.Tensor, targets: torch.Tensor):
    """eval.py:216-218: the CRPS of the averaged predictions under the model's loss."""
    return model.loss_fn.crps(preds, targets)
