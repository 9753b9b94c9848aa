"""The N>1 image-strip path on CPU: world_size-2 (and 3) gloo process groups, each rank
renders its interleaved bands (the oracle stands in for the GPU kernel here), one
all_gather of the padded local buffers, re-assembly on rank 0 -- must equal the
single-process render (imageUtils.h SSAA blocks stay inside bands)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, band, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch
    import torch.distributed as dist
    from raytracercpp_amd import scenes, strips
    from oracle.bindings import Oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc, st = scenes.robot1080(width=96, height=54, enable_ssaa=True, ssaa_factor=2)
    rw, rh = st.render_size()
    f = st.ssaa_factor
    o = Oracle(sc, st)
    rows = strips.rank_rows(st.image_height, band, rank, world)
    local = np.zeros((len(rows), st.image_width), np.uint32)
    for i, g in enumerate(rows):
        if g < 0:
            continue
        res = o.render_rows(g * f, f, nthreads=1)
        local[i] = Oracle.downscale(res.argb, rw, f, f)
    t = torch.from_numpy(local.view(np.int32).copy())
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    if rank == 0:
        img = strips.assemble([p.numpy().view(np.uint32) for p in parts], st.image_height, band)
        q.put(img)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,band", [(2, 8), (3, 5)])
def test_gloo_strips_equal_single_process(world, band):
    from raytracercpp_amd import scenes
    from oracle.bindings import Oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, band, q)) for r in range(world)]
    for p in procs:
        p.start()
    img = q.get(timeout=300)
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    sc, st = scenes.robot1080(width=96, height=54, enable_ssaa=True, ssaa_factor=2)
    rw, rh = st.render_size()
    full = Oracle(sc, st).render_rows()
    ref = Oracle.downscale(full.argb, rw, rh, 2).reshape(st.image_height, st.image_width)
    assert np.array_equal(img, ref)


def _pipe_worker(rank, world, port, nslots, nframes, q):
    """FramePipeline over gloo: frame k's strips of rank r hold (k, r, local row); every
    frame's gathered parts must be that frame's, in rank order, although the next
    frames are enqueued before it is read (slots are reused only after their gather)."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch
    import torch.distributed as dist
    from raytracercpp_amd.strips import FramePipeline
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    frame = [0]

    def render(out, stream):
        assert stream is None
        rows = torch.arange(out.shape[0], dtype=torch.int32).unsqueeze(1)
        out.copy_((frame[0] * 1000 + rank * 100 + rows).expand_as(out))
        frame[0] += 1

    outs = [torch.zeros((5, 7), dtype=torch.int32) for _ in range(nslots)]
    pipe = FramePipeline(render, outs, world, None, dist)
    seen = []
    for k in range(nframes):
        slot = pipe.step()
        if k >= nslots - 1:   # the frame enqueued nslots-1 steps ago has its gather in flight
            old = (slot + 1) % nslots
            if pipe.works[old] is not None:
                pipe.works[old].wait()
                pipe.works[old] = None
            seen.append([p.clone() for p in pipe.parts[old]])
    pipe.drain()
    ok = len(seen) == nframes - (nslots - 1)
    for k, parts in enumerate(seen):   # seen[k] was read at step k + nslots - 1: frame k
        for r, p in enumerate(parts):
            rows = torch.arange(5, dtype=torch.int32).unsqueeze(1)
            ok &= bool(torch.equal(p, (k * 1000 + r * 100 + rows).expand(5, 7)))
    last = (nframes - 1) % nslots
    for r, p in enumerate(pipe.parts[last]):
        rows = torch.arange(5, dtype=torch.int32).unsqueeze(1)
        ok &= bool(torch.equal(p, ((nframes - 1) * 1000 + r * 100 + rows).expand(5, 7)))
    q.put((rank, ok))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("nslots", [1, 2, 3])
def test_gloo_frame_pipeline(nslots):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, world, port, nslots, 7, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    assert all(ok for _, ok in res), res


@pytest.mark.parametrize("nranks", [1, 2, 3, 8])
def test_assign_bands_balanced_and_deterministic(nranks):
    """strips.assign_bands: every band exactly once, equal band counts (ceil or one fewer, so the
    all-gather keeps one buffer size), the same lists from the same vector, and the predicted loads
    within the costliest band of each other (longest processing time first); assemble with the
    lists re-builds the frame from per-rank buffers."""
    from raytracercpp_amd.strips import assemble, assign_bands, list_rows
    rng = np.random.default_rng(nranks)
    H, band = 1080, 8
    nb = (H + band - 1) // band
    costs = rng.exponential(size=nb) * (rng.random(nb) < 0.3) + 1e-3
    costs[60:67] *= 50.0   # a cluster of costly bands (the sphere's silhouette / pole rows)
    lists = assign_bands(costs, nranks)
    assert all(np.array_equal(a, b) for a, b in zip(lists, assign_bands(costs.copy(), nranks)))
    flat = np.concatenate(lists)
    assert sorted(flat.tolist()) == list(range(nb))
    per = (nb + nranks - 1) // nranks
    assert all(len(lst) in (per, per - 1) for lst in lists) and len(lists[0]) == per
    loads = np.array([costs[lst].sum() for lst in lists])
    assert loads.max() - loads.min() <= costs.max() + 1e-9
    W = 5
    frame = (np.arange(H)[:, None] * 7 + np.arange(W)[None]).astype(np.int32)
    parts = []
    for lst in lists:
        g = list_rows(lst, H, band, per)
        p = np.zeros((per * band, W), np.int32)
        p[g >= 0] = frame[g[g >= 0]]
        parts.append(p)
    assert np.array_equal(assemble(parts, H, band, lists), frame)
