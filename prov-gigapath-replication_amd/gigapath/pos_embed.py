"""2-D sin-cos position embedding, factorised for the MI355X path.

The reference materialises a [1 + G*G, E] fp32 table (gigapath/pos_embed.py:30-77; 3.07 GB at
G = 1000, E = 768) and gathers rows of it (slide_encoder.py:200).  Row p > 0 of that table is
the concatenation of two rows of ONE [G, E/2] table: the y index (p-1) % G for the first E/2
columns and the x index (p-1) // G for the last E/2 (``meshgrid(w, h)`` puts w first).  Both
halves are built here with the same fp64 numpy arithmetic and rounded once to fp32, so every
row is bit-identical to the reference buffer; the HIP kernel gp_posembed_cls_ln reads the
two half-rows directly.
"""
from __future__ import annotations

import numpy as np


def get_1d_sincos_pos_embed_from_grid(embed_dim: int, pos) -> np.ndarray:
    """[M, embed_dim] fp64: [sin(pos * w) | cos(pos * w)], w_k = 10000**(-2k/embed_dim)."""
    if embed_dim % 2:
        raise ValueError("embed_dim must be even")
    w = np.arange(embed_dim // 2, dtype=float)
    w /= embed_dim / 2.0
    w = 1.0 / 10000 ** w
    ang = np.einsum("m,d->md", np.asarray(pos).reshape(-1), w)
    return np.concatenate([np.sin(ang), np.cos(ang)], axis=1)


def axis_table(embed_dim: int, grid_size: int) -> np.ndarray:
    """The [G, E/2] fp32 half-row table (one grid axis)."""
    if embed_dim % 4:
        raise ValueError("embed_dim must be a multiple of 4")
    ticks = np.arange(grid_size, dtype=np.float32)
    return get_1d_sincos_pos_embed_from_grid(embed_dim // 2, ticks).astype(np.float32)


def get_2d_sincos_pos_embed(embed_dim: int, grid_size: int, cls_token: bool = False) -> np.ndarray:
    """Full table, API-compatible with the reference (used only when ``model.pos_embed`` is read)."""
    half = axis_table(embed_dim, grid_size).astype(np.float64)
    q = np.arange(grid_size * grid_size)
    full = np.concatenate([half[q % grid_size], half[q // grid_size]], axis=1)
    if cls_token:
        full = np.concatenate([np.zeros([1, embed_dim]), full], axis=0)
    return full
