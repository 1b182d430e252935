"""Drop-in ``NeRFSmall`` (models.py:96-174) on the gfx950 MFMA kernels."""
from __future__ import annotations

import torch
import torch.nn as nn

from . import functional as HF

SUPPORTED = dict(num_layers=2, hidden_dim=64, geo_feat_dim=15, num_layers_color=3,
                 hidden_dim_color=64, input_ch=32, input_ch_views=16)


class NeRFSmall(nn.Module):
    """sigma net 32->64->16, color net [sh16|geo15]->64->64->3; ReLU, no biases,
    no output activation; forward(x[N,48]) -> [N,4] = [rgb3 | sigma]."""

    def __init__(self, num_layers=3, hidden_dim=64, geo_feat_dim=15, num_layers_color=4,
                 hidden_dim_color=64, input_ch=3, input_ch_views=3):
        super().__init__()
        cfg = dict(num_layers=num_layers, hidden_dim=hidden_dim, geo_feat_dim=geo_feat_dim,
                   num_layers_color=num_layers_color, hidden_dim_color=hidden_dim_color,
                   input_ch=input_ch, input_ch_views=input_ch_views)
        if cfg != SUPPORTED:
            raise NotImplementedError(
                f"hashnerf_amd.NeRFSmall: only the create_nerf configuration {SUPPORTED} "
                "(run_nerf_helpers.py:79-84) has a HIP kernel")
        self.input_ch, self.input_ch_views = input_ch, input_ch_views
        self.num_layers, self.hidden_dim, self.geo_feat_dim = num_layers, hidden_dim, geo_feat_dim
        self.num_layers_color, self.hidden_dim_color = num_layers_color, hidden_dim_color
        self.sigma_net = nn.ModuleList([nn.Linear(input_ch, hidden_dim, bias=False),
                                        nn.Linear(hidden_dim, 1 + geo_feat_dim, bias=False)])
        self.color_net = nn.ModuleList([
            nn.Linear(input_ch_views + geo_feat_dim, hidden_dim_color, bias=False),
            nn.Linear(hidden_dim_color, hidden_dim_color, bias=False),
            nn.Linear(hidden_dim_color, 3, bias=False)])

    def weights(self):
        return [self.sigma_net[0].weight, self.sigma_net[1].weight, self.color_net[0].weight,
                self.color_net[1].weight, self.color_net[2].weight]

    def forward(self, x):
        return HF.NeRFSmallFn.apply(x, *self.weights())
