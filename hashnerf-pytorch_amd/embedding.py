"""Drop-in ``HashEmbedder`` / ``SHEncoder`` (embedding/hash_encoding.py,
embedding/spherical_harmonic.py) backed by the gfx950 HIP kernels.

Storage: the L per-level tables live in ONE contiguous parameter
``table [L, 2^T, F]`` (HBM layout the kernels read); ``embeddings[l]`` are
views of it with the reference's ``nn.Embedding`` calling convention, and the
state dict keeps the reference's keys ``embeddings.{l}.weight`` so checkpoints
round-trip (run_nerf.py:663-680, run_nerf_helpers.py:158-168).
"""
from __future__ import annotations

from typing import Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib as L
from . import functional as HF

HASH_PRIMES = [1, 2654435761, 805459861, 3674653429, 2097192037, 1434869437, 2165219737]


def level_resolutions(n_levels, base_resolution, finest_resolution):
    """fp32 ``floor(base * b**l)`` exactly as hash_encoding.py:46-50, :101."""
    base = torch.as_tensor(base_resolution)
    finest = torch.as_tensor(finest_resolution)
    b = torch.exp((torch.log(finest) - torch.log(base)) / (n_levels - 1))
    return b, [torch.floor(base * b ** i) for i in range(n_levels)]


def hash(coords: torch.Tensor, log2_hashmap_size: int) -> torch.Tensor:
    """Spatial hash of integer coords [..., d] (hash_encoding.py:112-128);
    host/torch helper used by the TV loss cube gather."""
    out = torch.zeros_like(coords[..., 0])
    for i in range(coords.shape[-1]):
        out ^= coords[..., i] * HASH_PRIMES[i]
    return out & ((1 << log2_hashmap_size) - 1)


class _LevelEmbedding(nn.Module):
    """``embeddings[l]``: an nn.Embedding-like view of one level of the table."""

    def __init__(self, owner: "HashEmbedder", level: int):
        super().__init__()
        object.__setattr__(self, "_owner", owner)   # not a registered submodule
        self.level = level

    @property
    def weight(self) -> torch.Tensor:
        return self._owner.table[self.level]

    @property
    def num_embeddings(self):
        return self._owner.table.shape[1]

    @property
    def embedding_dim(self):
        return self._owner.table.shape[2]

    def forward(self, idx: torch.Tensor) -> torch.Tensor:
        return F.embedding(idx, self.weight)

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        pass   # the owning HashEmbedder consumes embeddings.{l}.weight


class HashEmbedder(nn.Module):
    """Multiresolution hash encoding (hash_encoding.py:13-110)."""

    def __init__(self, bounding_box, n_levels=16, n_features_per_level=2,
                 log2_hashmap_size=19, base_resolution=16, finest_resolution=512):
        super().__init__()
        if n_features_per_level != 2:
            raise NotImplementedError("hashnerf_amd: n_features_per_level must be 2")
        if not (1 <= n_levels <= L.MAX_LEVELS):
            raise NotImplementedError(f"hashnerf_amd: n_levels must be in [1, {L.MAX_LEVELS}]")
        self.bounding_box = bounding_box
        self.n_levels = n_levels
        self.n_features_per_level = n_features_per_level
        self.log2_hashmap_size = log2_hashmap_size
        self.base_resolution = torch.tensor(base_resolution)
        self.finest_resolution = torch.tensor(finest_resolution)
        self.out_dim = n_levels * n_features_per_level
        self.b, self.resolutions = level_resolutions(n_levels, self.base_resolution,
                                                     self.finest_resolution)
        self.table = nn.Parameter(torch.empty(n_levels, 2 ** log2_hashmap_size,
                                              n_features_per_level))
        nn.init.uniform_(self.table, a=-0.0001, b=0.0001)            # :55-56
        # RAdam.state_dict / load_state_dict list this parameter as the
        # reference's n_levels per-level embedding weights
        self.table._hn_levels = n_levels
        self.embeddings = nn.ModuleList([_LevelEmbedding(self, l) for l in range(n_levels)])
        self._grid = None

    # -- geometry ---------------------------------------------------------
    def box(self):
        bmin, bmax = self.bounding_box
        return (torch.as_tensor(bmin, dtype=torch.float32).cpu(),
                torch.as_tensor(bmax, dtype=torch.float32).cpu())

    def grid(self) -> L.HnGrid:
        """hn_grid with fp32 cell sizes (box_max - box_min) / res_l (:72)."""
        if self._grid is None:
            bmin, bmax = self.box()
            gs = [((bmax - bmin) / r).tolist() for r in self.resolutions]
            self._grid = L.make_grid(self.n_levels, self.n_features_per_level,
                                     self.log2_hashmap_size, bmin.tolist(), bmax.tolist(), gs)
        return self._grid

    def forward(self, x: torch.Tensor):
        """x [N,3] -> (feat [N, L*F], keep_mask [N] bool)."""
        return HF.hash_encode(x, self.table, self.grid())

    # -- reference-compatible state dict: embeddings.{l}.weight ------------
    def _save_to_state_dict(self, destination, prefix, keep_vars):
        for l in range(self.n_levels):
            w = self.table[l]
            destination[prefix + f"embeddings.{l}.weight"] = w if keep_vars else w.detach()

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        for l in range(self.n_levels):
            k = prefix + f"embeddings.{l}.weight"
            if k in state_dict:
                with torch.no_grad():
                    self.table[l].copy_(state_dict[k])
            elif strict:
                missing_keys.append(k)
        if strict:
            for k in state_dict:
                if k.startswith(prefix) and k[len(prefix):].split(".")[0] not in ("embeddings",):
                    unexpected_keys.append(k)


class SHEncoder(nn.Module):
    """Real spherical harmonics of the view direction (spherical_harmonic.py:43-103)."""

    def __init__(self, input_dim=3, degree=4):
        super().__init__()
        assert input_dim == 3
        assert 1 <= degree <= 5
        if degree > 4:
            raise NotImplementedError("hashnerf_amd: SH degree 5 is not implemented (reference "
                                      "default and every config use degree 4)")
        self.input_dim = input_dim
        self.degree = degree
        self.out_dim = degree ** 2

    def forward(self, input, **kwargs):
        out = HF.sh_encode(input)
        return out if self.degree == 4 else out[..., : self.out_dim].contiguous()
