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


def num_bands(image_h: int, band_rows: int) -> int:
    return (image_h + band_rows - 1) // band_rows


def assign_bands(costs, nranks: int):
    """Cost-balanced strips: the bands (global indices) of each rank, from each band's cost in an
    earlier frame (rt_band_costs, summed over the ranks that rendered them).  Every rank gets the
    same number of bands, ceil(nb / nranks), or one fewer, so the local buffers and the all-gather
    keep one size; bands are dealt costliest first to the rank with the least predicted cost that
    still has room (longest processing time first), ties to the lower rank, so that every rank
    computes the same assignment from the same vector.  Each rank's list is sorted (row order)."""
    c = np.asarray(costs, np.float64)
    nb = c.size
    per = (nb + nranks - 1) // nranks
    cap = np.full(nranks, per, np.int64)
    cap[nranks - (per * nranks - nb):] -= 1   # the last per * nranks - nb ranks take one band fewer
    load = np.zeros(nranks)
    out = [[] for _ in range(nranks)]
    for b in np.lexsort((np.arange(nb), -c)):   # costliest first, then band order
        room = np.flatnonzero(np.array([len(o) for o in out]) < cap)
        r = int(room[np.argmin(load[room])])
        out[r].append(int(b))
        load[r] += c[b]
    return [np.array(sorted(o), np.int32) for o in out]


def interleaved_bands(image_h: int, band_rows: int, nranks: int):
    """The default layout as band lists: band b goes to rank b % nranks."""
    nb = num_bands(image_h, band_rows)
    return [np.arange(r, nb, nranks, dtype=np.int32) for r in range(nranks)]


def list_rows(bands, image_h: int, band_rows: int, local_bands: int) -> np.ndarray:
    """Global output row of each local row of a rank rendering ``bands`` into a buffer of
    ``local_bands`` bands (-1 for padding rows)."""
    g = np.full(local_bands * band_rows, -1, np.int64)
    for i, b in enumerate(bands):
        rows = b * band_rows + np.arange(band_rows)
        g[i * band_rows:(i + 1) * band_rows] = np.where(rows < image_h, rows, -1)
    return g


def _row_maps(nranks, image_h, band_rows, assignment, local_n):
    if assignment is None:
        return [rank_rows(image_h, band_rows, r, nranks) for r in range(nranks)]
    return [list_rows(assignment[r], image_h, band_rows, local_n // band_rows) for r in range(nranks)]


def assemble(parts, image_h: int, band_rows: int, assignment=None):
    """parts[r]: (local_rows, W) array of rank r -> (image_h, W) frame.  ``assignment``: the band
    list of each rank (assign_bands), or None for the interleaved layout."""
    nranks = len(parts)
    W = parts[0].shape[1]
    out = np.zeros((image_h, W), dtype=parts[0].dtype)
    for r, (p, g) in enumerate(zip(parts, _row_maps(nranks, image_h, band_rows, assignment, parts[0].shape[0]))):
        keep = g >= 0
        out[g[keep]] = np.asarray(p)[keep]
    return out


def assemble_torch(parts, image_h: int, band_rows: int, assignment=None):
    """Same as :func:`assemble` on torch tensors (stays on the device)."""
    import torch
    nranks = len(parts)
    W = parts[0].shape[1]
    out = torch.zeros((image_h, W), dtype=parts[0].dtype, device=parts[0].device)
    for p, g in zip(parts, _row_maps(nranks, image_h, band_rows, assignment, parts[0].shape[0])):
        g = torch.as_tensor(g, device=p.device)
        keep = g >= 0
        out[g[keep]] = p[keep]
    return out


def gather_index(image_h: int, band_rows: int, nranks: int, local_n: int, assignment=None) -> np.ndarray:
    """For the all-gathered buffer (nranks x local_n rows, rank-major): the row of each output row,
    so that frame = gathered[index] (the re-assembly as one device gather)."""
    idx = np.full(image_h, -1, np.int64)
    for r, g in enumerate(_row_maps(nranks, image_h, band_rows, assignment, local_n)):
        keep = np.flatnonzero(g >= 0)
        idx[g[keep]] = r * local_n + keep
    assert (idx >= 0).all(), "a row no rank renders"
    return idx


class FramePipeline:
    """Frames in flight over ``q`` slots.

    Step i uses slot i % q: its stream, its output buffer and its gather buffer.  The render is
    enqueued on the slot's stream and the all-gather of the slot's strips (one flat buffer, rank-major)
    is enqueued asynchronously behind it, so frame i's gather and tail overlap frame i+1's render on
    the other streams.  With ``assemble`` (rank 0), the slot's stream then waits for the gather and
    ``assemble(slot, gathered)`` re-assembles the frame there, inside the step (Renderer::get_image's
    whole image).  A slot is reused only after its previous gather has finished reading the buffer
    (``work.wait()``, which on a GPU makes the slot's stream wait and on CPU blocks).
    ``render(out, stream)`` writes one rank's strips into ``out``.  With ``streams=None`` (CPU / gloo)
    everything runs on the host in order.
    """

    def __init__(self, render, outs, world: int, streams=None, dist=None, assemble=None, gather=None):
        self.render = render
        self.outs = outs
        self.q = len(outs)
        self.world = world
        self.streams = streams
        self.dist = dist
        self.assemble = assemble
        self.gather = world > 1 if gather is None else gather   # (gather=True with one rank: tests)
        self.flat = [o.new_empty((world * o.shape[0],) + tuple(o.shape[1:])) for o in outs] if self.gather else None
        n = outs[0].shape[0]
        self.parts = ([[f[r * n:(r + 1) * n] for r in range(world)] for f in self.flat] if self.gather
                      else [[o] for o in outs])
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
            if self.gather:
                self.works[i] = self.dist.all_gather_into_tensor(self.flat[i], self.outs[i], async_op=True)
                if self.assemble is not None:
                    self.works[i].wait()
                    self.works[i] = None
                    self.assemble(i, self.flat[i])
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
