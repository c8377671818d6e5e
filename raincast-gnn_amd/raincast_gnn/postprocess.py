"""Output post-processing (models/model_utils.py:42-113), unchanged semantics.

softplus(.) + 1e-6 on the scale parameters, sigmoid on the point-mass probability and
``2.12 * sigmoid(u)`` for a learned threshold.  ``grad_u`` is the params.json STRING
compared with "True" (model_utils.py:99, Appendix A of SURVEY.md).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

EPS = 1e-6


class MakePositive(torch.nn.Module):
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        mu, sigma = torch.split(x, 1, dim=-1)
        return torch.cat([mu, F.softplus(sigma) + EPS], dim=-1)


class PostProcess(torch.nn.Module):
    def __init__(self, loss: str, grad_u):
        super().__init__()
        self.loss = loss
        self.grad_u = grad_u

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.loss == "NormalCRPS":
            return MakePositive()(x)
        if self.loss == "MixedNormalCRPS":
            mu, sigma, p = torch.split(x, 1, dim=-1)
            return torch.cat([mu, F.softplus(sigma) + EPS, F.sigmoid(p)], dim=-1)
        if self.loss == "MixedLoss":
            if self.grad_u == "True":
                mu, sigma, p, sigma_u, u = torch.split(x, 1, dim=-1)
                return torch.cat([mu, F.softplus(sigma) + EPS, F.sigmoid(p),
                                  F.softplus(sigma_u) + EPS, F.sigmoid(u) * 2.12], dim=-1)
            mu, sigma, p, sigma_u = torch.split(x, 1, dim=-1)
            return torch.cat([mu, F.softplus(sigma) + EPS, F.sigmoid(p),
                              F.softplus(sigma_u) + EPS], dim=-1)
        raise ValueError(f"unknown loss '{self.loss}'")
