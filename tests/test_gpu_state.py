"""Shim state across calls: frame pipelining's slot/stream ordering, the
process-wide device scene shared by several Raytracer instances, and
re-initialisation after rt_gpu_shutdown."""
import ctypes

import numpy as np
import pytest

import helpers
from test_gpu_parity import render_gpu

pytestmark = pytest.mark.gpu


def _params(scene, w, h, depth, ao, root):
    rt580 = helpers.rt580()
    rt = rt580.Raytracer(w, h, root)
    assert rt.LoadSceneJSON(scene) == 0
    rt.set_depth(depth)
    rt.set_ao(ao, True)
    assert rt.InitializeRenderer() == 0
    return rt, rt.render_params()


def test_pipelined_frames_alternating_accel_keep_each_framebuffer():
    """Consecutive frames alternate between two slots, BVH frames included;
    a frame must not overwrite a slot's framebuffer while work the caller
    queued against it (a delayed read on the caller's stream) is still
    pending (rt_shim.cpp begin_slot)."""
    import torch
    rt580 = helpers.rt580()
    lib = rt580.load()
    root = helpers.synthetic_root("cornell10k")
    w, h = 40, 24
    cfg = [(2, 4), (3, 8)]  # (depth, AO): the two alternating frames differ
    want = [render_gpu("cornell10k.json", w, h, d, a, True, root=root)[0] for d, a in cfg]
    rts = [_params("cornell10k.json", w, h, d, a, root) for d, a in cfg]
    s = rts[0][0].scene()
    rt580.check(lib.rt_gpu_upload_scene(ctypes.byref(s)), "upload")
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    rt580.check(lib.rt_gpu_set_stream(ctypes.c_void_p(stream.cuda_stream)), "stream")
    n = w * h * 3
    outs = []
    try:
        for i in range(8):
            k = i % 2
            assert lib.rt_gpu_set_accel(1 if k == 0 else 0) == 0  # BVH / brute force
            fbp = ctypes.c_void_p()
            rt580.check(lib.rt_gpu_render_device(ctypes.byref(rts[k][1]), ctypes.byref(fbp)), "render_device")
            torch.cuda._sleep(2_000_000)  # the caller's read of this frame's fb is late
            o = torch.empty(n, dtype=torch.uint8, device=dev)
            rt580.check(lib.rt_gpu_gamma_u8(fbp, n, o.data_ptr()), "gamma_u8")
            outs.append((k, o))
        torch.cuda.synchronize()
    finally:
        lib.rt_gpu_set_accel(1)
        lib.rt_gpu_set_stream(lib.rt_gpu_own_stream())
    for i, (k, o) in enumerate(outs):
        body = rt580.ppm_bytes(want[k]).split(b"\n", 3)[3]
        assert o.cpu().numpy().tobytes() == body, "frame %d (config %d) was overwritten" % (i, k)


def test_two_instances_with_different_scenes_interleave():
    """The device scene is process-wide: instance A must re-upload its scene
    after instance B rendered another one (raytracer.cpp Render)."""
    rt580 = helpers.rt580()
    a = rt580.Raytracer(48, 36, helpers.ASSETS_ROOT)
    b = rt580.Raytracer(48, 36, helpers.ASSETS_ROOT)
    assert a.LoadSceneJSON("simpleSphereScene.json") == 0 and b.LoadSceneJSON("scene.json") == 0
    for r in (a, b):
        r.set_depth(2)
        r.set_ao(4, True)
    assert a.Render("") == 0
    fa = a.framebuffer()
    assert b.Render("") == 0
    fb = b.framebuffer()
    assert a.Render("") == 0
    assert np.array_equal(a.framebuffer(), fa)
    assert b.Render("") == 0
    assert np.array_equal(b.framebuffer(), fb)
    assert not np.array_equal(fa, fb)
    # after a shutdown the next Render initialises and uploads again
    rt580.load().rt_gpu_shutdown()
    assert a.Render("") == 0
    assert np.array_equal(a.framebuffer(), fa)
    ref, _ = helpers.oracle_render("simpleSphereScene.json", 48, 36, 2, 4, True)
    assert np.array_equal(fa, ref)
    a.close()
    b.close()


def test_count_rows_then_full_render_same_params():
    """rt_gpu_count_rows traces only the selected rows, rt_gpu_render the
    prefix; the node-capacity verification must not carry over between them
    (rt_shim.cpp check_capacity keys on the traced rows)."""
    import torch
    rt580 = helpers.rt580()
    lib = rt580.load()
    d = helpers.rt580_dist()
    scene, w, h, depth, ao = "simpleSphereSceneAO.json", 64, 48, 8, 4
    rt, params = _params(scene, w, h, depth, ao, helpers.ASSETS_ROOT)
    s = rt.scene()
    rt580.check(lib.rt_gpu_upload_scene(ctypes.byref(s)), "upload")
    dev = torch.device("cuda", 0)
    rt580.check(lib.rt_gpu_set_stream(ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "stream")
    try:
        d.GpuRows(rt580, params, torch, dev).count(0, 4)
        torch.cuda.synchronize()
        host = np.zeros(w * h * 3, dtype=np.int16)
        rt580.check(lib.rt_gpu_render(ctypes.byref(params), host.ctypes.data), "render")
    finally:
        lib.rt_gpu_set_stream(lib.rt_gpu_own_stream())
    ref, _ = helpers.oracle_render(scene, w, h, depth, ao, True)
    assert np.array_equal(host.reshape(h, w, 3), ref)


def _device_frames(lib, rt580, seq, n, dev, torch):
    """rt_gpu_render_device for each params in seq, without a host sync in
    between; each frame's gamma-mapped bytes copied on the caller's stream."""
    outs = []
    for prm in seq:
        fbp = ctypes.c_void_p()
        rt580.check(lib.rt_gpu_render_device(ctypes.byref(prm), ctypes.byref(fbp)), "render_device")
        o = torch.empty(n, dtype=torch.uint8, device=dev)
        rt580.check(lib.rt_gpu_gamma_u8(fbp, n, o.data_ptr()), "gamma_u8")
        outs.append(o)
    torch.cuda.synchronize()
    return [o.cpu().numpy().tobytes() for o in outs]


def test_replayed_bvh_frames_match_oracle():
    """Repeats of a verified BVH frame replay its recorded host reads (count
    schedule, rt_shim.cpp trace_rows / shade_rows) and enqueue without a host
    sync, overlapping on the two slots. Many chunks per pass (chunk limit
    2^8), two interleaved configurations, a chunk-limit change in between
    (new key: recorded again): every frame equals the CPU restatement."""
    import torch
    rt580 = helpers.rt580()
    lib = rt580.load()
    root = helpers.synthetic_root("cornell10k")
    w, h = 48, 27
    cfg = [(4, 16), (2, 8)]
    want = []
    for d, a in cfg:
        ref, _ = helpers.oracle_render("cornell10k.json", w, h, d, a, True, root=root)
        want.append(rt580.ppm_bytes(ref).split(b"\n", 3)[3])
    rts = [_params("cornell10k.json", w, h, d, a, root) for d, a in cfg]
    s = rts[0][0].scene()
    rt580.check(lib.rt_gpu_upload_scene(ctypes.byref(s)), "upload")
    dev = torch.device("cuda", 0)
    rt580.check(lib.rt_gpu_set_stream(ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "stream")
    n = w * h * 3
    order = [0, 0, 0, 0, 1, 1, 1, 0, 1, 0]
    try:
        for log2 in (8, 27):
            assert lib.rt580_set_chunk_log2(log2) == 0
            got = _device_frames(lib, rt580, [rts[k][1] for k in order], n, dev, torch)
            assert lib.rt_gpu_accel_active() == 1
            for i, (k, b) in enumerate(zip(order, got)):
                assert b == want[k], "frame %d (config %d, chunk 2^%d) differs" % (i, k, log2)
        # the synchronous path checks the replayed counts of its own frame
        host = np.zeros(n, dtype=np.int16)
        for _ in range(3):
            rt580.check(lib.rt_gpu_render(ctypes.byref(rts[0][1]), host.ctypes.data), "render")
    finally:
        lib.rt580_set_chunk_log2(27)
        lib.rt_gpu_set_stream(lib.rt_gpu_own_stream())


_CORRUPT_CHILD = r"""
import ctypes, sys
sys.path.insert(0, sys.argv[1])
import helpers
rt580 = helpers.rt580()
lib = rt580.load()
rt = rt580.Raytracer(48, 27, helpers.synthetic_root("cornell10k"))
assert rt.LoadSceneJSON("cornell10k.json") == 0
rt.set_depth(2)
rt.set_ao(8, True)
codes = [rt.Render("") for _ in range(4)]
print("CODES", codes, lib.rt_gpu_last_error().decode() if isinstance(lib.rt_gpu_last_error(), bytes) else lib.rt_gpu_last_error())
"""


def test_replay_count_mismatch_fails_the_frame(tmp_path):
    """Diagnostic build, RT580_REPLAY_CORRUPT=1: every replayed count's device
    check fails. The second identical Render replays the trace counts (the
    first verified them) and must fail with the schedule error instead of
    returning a frame; the schedules are dropped, so the third records again
    (succeeds) and the fourth replays both phases (fails)."""
    import os
    import subprocess
    import sys
    diag = os.path.join(helpers.REPO, "580-raytracer_amd", "lib580rt_diag.so")
    if not os.path.exists(diag):
        pytest.skip("diagnostic build absent (make diag)")
    env = dict(os.environ, RT580_LIB=diag, RT580_REPLAY_CORRUPT="1")
    script = tmp_path / "child.py"
    script.write_text(_CORRUPT_CHILD)
    r = subprocess.run([sys.executable, str(script), os.path.dirname(os.path.abspath(__file__))], env=env,
                       capture_output=True, text=True, timeout=240)
    line = [l for l in r.stdout.splitlines() if l.startswith("CODES")]
    assert line, r.stdout + r.stderr
    assert line[0].startswith("CODES [0, 1, 0, 1]"), line[0]
    assert "replayed count schedule" in line[0], line[0]
    # the device check names the count that differed (schedule, index, launcher step, both values)
    assert "first mismatch: count #" in line[0] and "recorded" in line[0], line[0]


_INFLATE_CHILD = r"""
import ctypes, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import helpers
rt580 = helpers.rt580()
lib = rt580.load()
rt = rt580.Raytracer(96, 54, helpers.synthetic_root("cornell10k"))
assert rt.LoadSceneJSON("cornell10k.json") == 0
rt.set_depth(2)
rt.set_ao(16, True)
codes, errs = [], []
for k in range(6):
    codes.append(rt.Render(""))
    e = lib.rt_gpu_last_error()
    errs.append(e.decode() if isinstance(e, bytes) else str(e))
    if codes[-1] == 0:
        np.save(sys.argv[2], rt.framebuffer())
print("CODES", codes)
for e in errs:
    print("ERR", e)
"""


def test_replayed_segment_count_inflated_fails_without_fault(tmp_path):
    """Diagnostic build, RT580_REPLAY_CORRUPT=2: a replayed far-queue segment
    count is replaced by a larger one (the queue length), so the launches after
    it are sized past the frame's segments and would read stale queue entries
    (round 5's illegal memory access: far_chunk_expand_kernel wrote work items
    past far_work from those entries' chunk counts). Every replayed frame must
    end as RT_FAILURE naming the count, with no device fault: the process
    keeps rendering, and the frames that record again equal the oracle's."""
    import os
    import subprocess
    import sys
    diag = os.path.join(helpers.REPO, "580-raytracer_amd", "lib580rt_diag.so")
    if not os.path.exists(diag):
        pytest.skip("diagnostic build absent (make diag)")
    env = dict(os.environ, RT580_LIB=diag, RT580_REPLAY_CORRUPT="2")
    script = tmp_path / "child.py"
    script.write_text(_INFLATE_CHILD)
    last = tmp_path / "last.npy"
    r = subprocess.run([sys.executable, str(script), os.path.dirname(os.path.abspath(__file__)), str(last)], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    line = [l for l in r.stdout.splitlines() if l.startswith("CODES")]
    assert line, r.stdout + r.stderr
    codes = eval(line[0][len("CODES "):])
    errs = [l[4:] for l in r.stdout.splitlines() if l.startswith("ERR ")]
    # the first frame records; every frame that replays the AO schedule fails (then records again)
    assert set(codes) <= {0, 1} and codes[0] == 0 and codes.count(1) >= 2 and codes[-1] == 0, (codes, errs)
    failed = [e for c, e in zip(codes, errs) if c == 1]
    assert all("replayed count schedule" in e for e in failed), failed
    assert any("far queue segments" in e for e in failed), failed
    assert not any("illegal" in e or "fault" in e.lower() for e in errs), errs
    assert "recorded" in failed[0] and "this frame" in failed[0]
    ref, _ = helpers.oracle_render("cornell10k.json", 96, 54, 2, 16, True, root=helpers.synthetic_root("cornell10k"))
    assert np.array_equal(np.load(last), ref), "the last recorded frame differs from the oracle"


def test_accel_toggle_on_repeated_frame_keeps_rendering():
    """The same params on a resident BVH scene, rendered (verified, recorded),
    then again (replayed), then under RT_ACCEL_BRUTE and back under AUTO: the
    recorded count schedules belong to the acceleration mode (rt_shim.cpp
    SchedKey.accel), so no toggle makes a frame fail, and every frame equals
    the oracle's."""
    rt580 = helpers.rt580()
    lib = rt580.load()
    root = helpers.synthetic_root("cornell10k")
    w, h, depth, ao = 40, 24, 3, 8
    rt, params = _params("cornell10k.json", w, h, depth, ao, root)
    s = rt.scene()
    rt580.check(lib.rt_gpu_upload_scene(ctypes.byref(s)), "upload")
    ref, _ = helpers.oracle_render("cornell10k.json", w, h, depth, ao, True, root=root)
    host = np.zeros(w * h * 3, dtype=np.int16)
    try:
        for mode in (1, 1, 0, 0, 1, 1, 0, 1):
            assert lib.rt_gpu_set_accel(mode) == 0
            rt580.check(lib.rt_gpu_render(ctypes.byref(params), host.ctypes.data), "render (accel %d)" % mode)
            assert lib.rt_gpu_accel_active() == mode
            assert np.array_equal(host.reshape(h, w, 3), ref), "accel %d" % mode
    finally:
        lib.rt_gpu_set_accel(1)
    rt.close()


def _registered(n_val):
    """A page-aligned, page-rounded int16 host buffer of n_val values (a
    registration must not share pages with other allocations)."""
    span = (n_val * 2 + 4095) // 4096 * 4096
    raw = np.zeros(span + 4096, dtype=np.uint8)
    off = (-raw.ctypes.data) % 4096
    return raw, raw[off:off + span].view(np.int16)[:n_val], span


def test_graph_replayed_small_frames_match_oracle():
    """The blocking small-scene rt_gpu_render into a registered framebuffer
    (render_split) runs each slot's frame as a HIP graph from the slot's second
    identical call on (rt_shim.cpp FrameGraph). Every call -- plain, captured,
    replayed, after a parameter change (new key) and into another registered
    buffer (new key) -- equals the CPU restatement."""
    rt580 = helpers.rt580()
    lib = rt580.load()
    scene, w, h = "simpleSphereSceneAO.json", 64, 48
    cfg = [(4, 8), (3, 4)]
    want = [helpers.oracle_render(scene, w, h, d, a, True)[0] for d, a in cfg]
    rts = [_params(scene, w, h, d, a, helpers.ASSETS_ROOT) for d, a in cfg]
    s = rts[0][0].scene()
    rt580.check(lib.rt_gpu_upload_scene(ctypes.byref(s)), "upload")
    bufs = [_registered(w * h * 3) for _ in range(2)]
    for _, buf, span in bufs:
        rt580.check(lib.rt_gpu_host_register(buf.ctypes.data, span), "host_register")
    try:
        # (config, buffer) per call: 6 calls cover plain, capture and replay on both slots
        for k, b in [(0, 0)] * 6 + [(1, 0)] * 5 + [(0, 1)] * 5 + [(0, 0)] * 2:
            buf = bufs[b][1]
            buf[:] = -1
            rt580.check(lib.rt_gpu_render(ctypes.byref(rts[k][1]), buf.ctypes.data), "render")
            assert np.array_equal(buf.reshape(h, w, 3), want[k]), "config %d buffer %d differs" % (k, b)
        # the captured graphs go with a shutdown; a fresh context captures its own
        lib.rt_gpu_shutdown()
        rt580.check(lib.rt_gpu_init(0), "init")
        rt580.check(lib.rt_gpu_upload_scene(ctypes.byref(s)), "upload")
        for _ in range(5):
            buf = bufs[0][1]
            buf[:] = -1
            rt580.check(lib.rt_gpu_render(ctypes.byref(rts[0][1]), buf.ctypes.data), "render after re-init")
            assert np.array_equal(buf.reshape(h, w, 3), want[0])
    finally:
        for _, buf, _ in bufs:
            lib.rt_gpu_host_unregister(buf.ctypes.data)


def test_last_stats_follow_graph_replayed_frames():
    """rt_gpu_last_stats after graph-replayed frames: frame A
    rendered into a registered buffer (plain, captured, replayed), then a
    different frame B left in HBM (rt_gpu_render_device), then A replayed
    again -- the counters always describe the frame just rendered."""
    rt580 = helpers.rt580()
    lib = rt580.load()
    scene, w, h = "simpleSphereSceneAO.json", 64, 48
    ra, pa = _params(scene, w, h, 4, 8, helpers.ASSETS_ROOT)
    rb, pb = _params(scene, 40, 24, 3, 4, helpers.ASSETS_ROOT)
    s = ra.scene()
    rt580.check(lib.rt_gpu_upload_scene(ctypes.byref(s)), "upload")
    keys = ("rays_total", "rays_primary", "rays_secondary", "rays_shadow", "rays_ao", "ao_calls")

    def stats():
        st = rt580.RenderStats()
        rt580.check(lib.rt_gpu_last_stats(ctypes.byref(st)), "last_stats")
        return tuple(getattr(st, k) for k in keys)

    raw, buf, span = _registered(w * h * 3)
    rt580.check(lib.rt_gpu_host_register(buf.ctypes.data, span), "host_register")
    try:
        rt580.check(lib.rt_gpu_render(ctypes.byref(pa), buf.ctypes.data), "render A")
        want_a = stats()
        assert want_a[1] == w * h and want_a[5] > 0
        for i in range(3):  # the slot's second identical call captures, later ones replay
            rt580.check(lib.rt_gpu_render(ctypes.byref(pa), buf.ctypes.data), "render A")
            assert stats() == want_a, "call %d" % i
        fb = ctypes.c_void_p()
        rt580.check(lib.rt_gpu_render_device(ctypes.byref(pb), ctypes.byref(fb)), "render_device B")
        rt580.check(lib.rt_gpu_synchronize(), "synchronize")
        want_b = stats()
        assert want_b[1] == 40 * 24 and want_b != want_a
        for i in range(2):
            rt580.check(lib.rt_gpu_render(ctypes.byref(pa), buf.ctypes.data), "render A again")
            assert stats() == want_a, "after B, call %d" % i
    finally:
        lib.rt_gpu_host_unregister(buf.ctypes.data)


_GRID_CHILD = r"""
import sys
sys.path.insert(0, sys.argv[1])
import numpy as np
import helpers
rt580 = helpers.rt580()
root = helpers.synthetic_root(sys.argv[2])
ok = []
for d, a in [(4, 16), (2, 8)]:
    rt = rt580.Raytracer(64, 36, root)
    assert rt.LoadSceneJSON(sys.argv[2] + ".json") == 0
    rt.set_depth(d)
    rt.set_ao(a, True)
    assert rt.Render("") == 0
    ref, _ = helpers.oracle_render(sys.argv[2] + ".json", 64, 36, d, a, True, root=root)
    ok.append(bool(np.array_equal(rt.framebuffer(), ref)))
    rt.close()
print("MATCH", ok)
"""


@pytest.mark.parametrize("scene", ["cornell10k", "field100k"])
def test_fine_direction_grid_small_frames_match_oracle(tmp_path, scene):
    """Frames below RT580_GRID_COARSE_PX pixels (every other GPU test's frame)
    take the half-resolution direction grid; the fine grid is the whole
    1080p-and-up frames'. RT580_GRID_COARSE_PX=0 forces the fine grid onto
    small frames: both grids answer as the oracle."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, RT580_GRID_COARSE_PX="0")
    script = tmp_path / "child.py"
    script.write_text(_GRID_CHILD)
    r = subprocess.run([sys.executable, str(script), os.path.dirname(os.path.abspath(__file__)), scene], env=env,
                       capture_output=True, text=True, timeout=280)
    line = [l for l in r.stdout.splitlines() if l.startswith("MATCH")]
    assert line, r.stdout + r.stderr
    assert line[0] == "MATCH [True, True]", line[0]


def test_render_async_frames_land_in_registered_buffers():
    """rt_gpu_render_async (the bench's N = 1 step): frames queued with their
    D2H copies into registered host buffers, several in flight, two
    configurations interleaved over a ring of buffers -- after a synchronize
    every buffer holds the last frame queued into it, equal to the oracle's; an
    unregistered buffer is refused."""
    rt580 = helpers.rt580()
    lib = rt580.load()
    root = helpers.synthetic_root("cornell10k")
    w, h = 48, 27
    cfg = [(4, 8), (2, 4)]
    want = [helpers.oracle_render("cornell10k.json", w, h, d, a, True, root=root)[0] for d, a in cfg]
    rts = [_params("cornell10k.json", w, h, d, a, root) for d, a in cfg]
    s = rts[0][0].scene()
    rt580.check(lib.rt_gpu_upload_scene(ctypes.byref(s)), "upload")
    bufs = [_registered(w * h * 3) for _ in range(3)]
    for _, buf, span in bufs:
        rt580.check(lib.rt_gpu_host_register(buf.ctypes.data, span), "host_register")
    try:
        last = {}
        for _, buf, _ in bufs:
            buf[:] = -1
        for i in range(11):
            k, b = i % 2, i % 3
            rt580.check(lib.rt_gpu_render_async(ctypes.byref(rts[k][1]), bufs[b][1].ctypes.data), "render_async")
            last[b] = k
        rt580.check(lib.rt_gpu_synchronize(), "synchronize")
        for b, k in last.items():
            assert np.array_equal(bufs[b][1].reshape(h, w, 3), want[k]), "buffer %d (config %d)" % (b, k)
        plain = np.zeros(w * h * 3, dtype=np.int16)
        assert lib.rt_gpu_render_async(ctypes.byref(rts[0][1]), plain.ctypes.data) != 0
    finally:
        for _, buf, _ in bufs:
            lib.rt_gpu_host_unregister(buf.ctypes.data)
    rts[0][0].close()
    rts[1][0].close()



def test_ao_audit_of_the_product_trace_and_late_passes(tmp_path):
    """Diagnostic build, RT580_AO_VERIFY=1 (rt_kernels.hip ao_audit_*): on the
    north-star frame, every near-query AO ray is answered again by the
    unbudgeted query, and the occlusion counts and far queue that implies are
    compared with what ao_trace_kernel / ao_late_kernel wrote -- their code is
    the product's (the audit adds kernels only): the budgeted speculative walk,
    the saved walks resumed by the late pass, and the late pass's re-read ray
    record (round 5: a 64-VGPR build of it, since removed, queued origins not
    their own when the origin stayed live across the walk)."""
    import json
    import os
    import subprocess
    import sys
    diag = os.path.join(helpers.REPO, "580-raytracer_amd", "lib580rt_diag.so")
    if not os.path.exists(diag):
        pytest.skip("diagnostic build absent (make diag)")
    env = dict(os.environ, RT580_LIB=diag, RT580_AO_VERIFY="1")
    r = subprocess.run([sys.executable, os.path.join(helpers.REPO, "tools", "ao_verify.py"), "field100k_1080p", "2"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    v = res["verify"]
    assert v["ok"] and v["entries_unexplained"] == 0 and v["rays_checked"] > 2e8, v
    assert res["frames_agree"] and not res["replay_errors"], res
    # the oracle's render of the whole frame (tests/golden/fullframe.json, make_fullframe.py)
    want = json.load(open(os.path.join(helpers.REPO, "tests", "golden", "fullframe.json")))["north_star"]["sha256"]
    assert res["hashes"][0] == want, res["hashes"]
