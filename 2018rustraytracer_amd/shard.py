"""Multi-GPU decomposition of the render path.

One process per GPU.  Two decompositions:

* frames (default bench mode): the orbiting-sphere animation is a sequence of
  independent frames (main.rs:1469); rank r renders frames r, r+N, r+2N, ...
  No data-path collective.

* row bands + gather: one frame is split into N contiguous row bands of
  ceil(H/N) rows (the last band may be short); every rank renders its band
  with RTM_FLAG_FUSED_SHADOW (each hit pixel evaluates the one shadow texel it
  reads, so no rank needs another rank's shadow map), then ONE gather
  (RCCL over xGMI on GPUs, gloo in the CPU tests) assembles the RGBA f32
  frame on rank 0.  Bands are padded to equal size so the gather is a single
  fixed-size collective; rank 0 views the first H rows of the padded result.
"""
from __future__ import annotations

from typing import List, Tuple


def band_rows(height: int, world: int) -> int:
    return (height + world - 1) // world


def row_band(height: int, world: int, rank: int) -> Tuple[int, int]:
    b = band_rows(height, world)
    return min(height, rank * b), min(height, (rank + 1) * b)


def row_bands(height: int, world: int) -> List[Tuple[int, int]]:
    return [row_band(height, world, r) for r in range(world)]


def stripe_rows_of(height: int, world: int, stripe: int, rank: int) -> int:
    """Rows of rank `rank` under `stripe`-row cyclic stripes (stripe j -> rank j % world);
    mirrors rtm_stripe_rows / rtm_api.cpp stripe_rows_of."""
    full, tail = divmod(height, stripe)
    rows = (full // world + (1 if rank < full % world else 0)) * stripe
    if tail and full % world == rank:
        rows += tail
    return rows


def stripe_image_rows(height: int, world: int, stripe: int, rank: int) -> List[int]:
    """The image rows of rank `rank`'s stripes, in its local (compact) order."""
    return [y for j in range(rank, (height + stripe - 1) // stripe, world)
            for y in range(j * stripe, min((j + 1) * stripe, height))]


def frames_for_rank(n_frames: int, rank: int, world: int) -> List[int]:
    return list(range(rank, n_frames, world))


def gather_bands(band, rank: int, world: int, height: int, dist, async_op: bool = False):
    """Gather equal-size padded bands (torch tensors [band_rows, W, C]) to rank 0.

    Returns (work, assembled): `assembled` is a [height, W, C] view on rank 0
    (None elsewhere) that is valid once `work` (None if synchronous) completes."""
    import torch

    if world == 1:
        return None, band[:height]
    if rank == 0:
        full = torch.empty((band.shape[0] * world,) + tuple(band.shape[1:]), dtype=band.dtype,
                           device=band.device)
        parts = list(full.chunk(world, dim=0))
        work = dist.gather(band, parts, dst=0, async_op=async_op)
        return work, full[:height]
    work = dist.gather(band, None, dst=0, async_op=async_op)
    return work, None
