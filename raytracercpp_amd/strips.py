"""Image-strip sharding across GPUs (one process per GPU).

Every output row of Renderer::ray_trace is independent (renderer.cpp:1082-1115) and
the SSAA box filter only mixes rows inside one ssaa_factor-row block
(imageUtils.h:121-146), so the frame is cut into bands of ``band_rows`` output
rows dealt round-robin to the ranks: band b goes to rank b % nranks.  Interleaved
bands balance the load (the object sits in the middle of the frame).  Each rank
renders its bands into a padded local buffer of ``local_rows`` rows; one
all-gather of those buffers (RCCL over xGMI, or gloo on CPU) is the only
collective, after which the frame is re-assembled by the row map below.
This mirrors the kernel's ``global_row`` (kernels.hip) and ``Renderer::local_rows``.
"""
from __future__ import annotations

import numpy as np


def local_rows(image_h: int, band_rows: int, nranks: int) -> int:
    nb = (image_h + band_rows - 1) // band_rows
    per = (nb + nranks - 1) // nranks
    return per * band_rows


def rank_rows(image_h: int, band_rows: int, rank: int, nranks: int) -> np.ndarray:
    """Global output row of each local row of ``rank`` (-1 for padding rows)."""
    n = local_rows(image_h, band_rows, nranks)
    lr = np.arange(n)
    band = lr // band_rows
    g = (band * nranks + rank) * band_rows + (lr - band * band_rows)
    g[g >= image_h] = -1
    return g


def assemble(parts, image_h: int, band_rows: int):
    """parts[r]: (local_rows, W) array of rank r -> (image_h, W) frame."""
    nranks = len(parts)
    W = parts[0].shape[1]
    out = np.zeros((image_h, W), dtype=parts[0].dtype)
    for r, p in enumerate(parts):
        g = rank_rows(image_h, band_rows, r, nranks)
        keep = g >= 0
        out[g[keep]] = np.asarray(p)[keep]
    return out


def assemble_torch(parts, image_h: int, band_rows: int):
    """Same as :func:`assemble` on torch tensors (stays on the device)."""
    import torch
    nranks = len(parts)
    W = parts[0].shape[1]
    out = torch.zeros((image_h, W), dtype=parts[0].dtype, device=parts[0].device)
    for r, p in enumerate(parts):
        g = torch.as_tensor(rank_rows(image_h, band_rows, r, nranks), device=p.device)
        keep = g >= 0
        out[g[keep]] = p[keep]
    return out


class FramePipeline:
    """Frames in flight over ``q`` slots.

    Step i uses slot i % q: its stream, its output buffer and its gather buffers.  The
    render is enqueued on the slot's stream and the all-gather of the slot's strips is
    enqueued asynchronously behind it, so frame i's gather and tail overlap frame i+1's
    render on the other stream.  A slot is reused only after its previous gather has
    finished reading the buffer (``work.wait()``, which on a GPU makes the slot's stream
    wait and on CPU blocks).  ``render(out, stream)`` writes one rank's strips into ``out``.
    With ``streams=None`` (CPU / gloo) everything runs on the host in order.
    """

    def __init__(self, render, outs, world: int, streams=None, dist=None):
        self.render = render
        self.outs = outs
        self.q = len(outs)
        self.world = world
        self.streams = streams
        self.dist = dist
        self.parts = [[o.new_empty(o.shape) for _ in range(world)] if world > 1 else [o] for o in outs]
        self.works = [None] * self.q
        self.count = 0

    def _ctx(self, i):
        import contextlib
        if self.streams is None:
            return contextlib.nullcontext()
        import torch
        return torch.cuda.stream(self.streams[i])

    def step(self) -> int:
        """Enqueue one frame; returns its slot."""
        i = self.count % self.q
        self.count += 1
        with self._ctx(i):
            if self.works[i] is not None:
                self.works[i].wait()
                self.works[i] = None
            self.render(self.outs[i], None if self.streams is None else self.streams[i])
            if self.world > 1:
                self.works[i] = self.dist.all_gather(self.parts[i], self.outs[i], async_op=True)
        return i

    def drain(self):
        """Wait for every enqueued frame and gather."""
        for i in range(self.q):
            if self.works[i] is not None:
                with self._ctx(i):
                    self.works[i].wait()
                self.works[i] = None
        if self.streams is not None:
            import torch
            torch.cuda.synchronize()
