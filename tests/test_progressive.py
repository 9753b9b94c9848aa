"""Progressive image readback (Renderer::lock_image_mutex / unlock_image_mutex, renderer.h:41-42;
DisplayThread::run polling get_image while RenderThread::run renders, QT/mainWindowThreads.cpp:6-65).

A display thread calls rt_get_image while the owning thread renders: it is not blocked by the
frame, it sees the internal-size image of the frame in progress (finished tiles over the
BACKGROUND_COLOR fill of a re-created SSAA image), and after post_process the downscaled final
image.  The image lock holds back a frame's switch of the image."""
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BG = 0xFF87CEEB   # BACKGROUND_COLOR (135, 206, 235) as ARGB32 (renderer.cpp:131-134)


@pytest.fixture(scope="module")
def R():
    from raytracercpp_amd.renderer import Renderer
    r = Renderer(0)
    yield r
    r.close()


def test_display_thread_sees_frame_in_progress():
    """C5 (rough reflections) with reflection chunks of 2^18 sample slots, so that level 1 writes
    its pixels chunk by chunk over the frame: snapshots taken while rt_render runs on another thread
    return in milliseconds, have the internal size, and show a partly rendered frame (some pixels
    already the frame's final ones, others not yet)."""
    import os
    from raytracercpp_amd import scenes
    from raytracercpp_amd.renderer import Renderer, render
    os.environ["RT_REFL_CHUNK_LOG2"] = "18"   # read once, at rt_create
    try:
        R = Renderer(0)
    finally:
        os.environ.pop("RT_REFL_CHUNK_LOG2")
    try:
        sc, st = scenes.sphere1m_refl(width=960, height=540)
        R.load_scene(sc, st)
        R.finish_accel()
        R.request_aux(rgba=False, hit=False, shadow=False)
        render(R)                       # warm: buffers sized, kernels loaded
        final_prev = R.get_image().copy()
        rw, rh = st.render_size()
        done = threading.Event()
        err = []

        def render_thread():
            try:
                render(R)
            except Exception as e:   # surfaced by the main thread
                err.append(e)
            done.set()

        snaps = []
        t = threading.Thread(target=render_thread)
        t.start()
        while not done.is_set():
            t0 = time.perf_counter()
            img = R.get_image()
            dt = time.perf_counter() - t0
            snaps.append((done.is_set(), img.shape, dt, img))
            time.sleep(0.002)
        t.join(120)
        assert not err, err
        final = R.get_image()
        assert final.shape == (st.image_height, st.image_width)
        assert np.array_equal(final, final_prev)   # the same frame again (path-keyed streams)
        internal = R.get_internal(argb=True)["argb"].reshape(rh, rw)
        inflight = [s for s in snaps if not s[0] and s[1] == (rh, rw)]
        assert len(inflight) >= 3, [(s[0], s[1], round(s[2], 4)) for s in snaps]
        # a snapshot does not wait for the frame
        assert min(s[2] for s in inflight) < 0.05, sorted(s[2] for s in inflight)[:5]
        obj = internal != BG   # the sphere's pixels
        partial = [s for s in inflight if 0 < int((s[3] == internal)[obj].sum()) < int(obj.sum())]
        assert partial, "no snapshot of a partly rendered frame"
    finally:
        R.close()


def test_image_lock_holds_back_the_frame(R):
    """While another thread holds the image lock, a frame does not start (its image switch
    waits); releasing the lock lets it finish."""
    from raytracercpp_amd import scenes
    sc, st = scenes.sphere256(width=64, height=64)
    R.load_scene(sc, st)
    R.ray_trace()
    done = threading.Event()
    R.lock_image()
    try:
        t = threading.Thread(target=lambda: (R.ray_trace(), done.set()))
        t.start()
        assert not done.wait(0.3)
        img = R.get_image()           # the lock is recursive: the holder still reads the image
        assert img.shape == (64, 64)
    finally:
        R.unlock_image()
    t.join(30)
    assert done.is_set()
