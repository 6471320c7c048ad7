"""Row-interleaved multi-rank rendering of one frame.

One process per GPU. Rank r of G renders rows r, r+G, r+2G, ... (interleaved
rows balance the work: sky rows are cheap). The reference draws every AO sample
from ONE serial RNG stream in raster order (Raytracer.h:592, Raytracer.cpp:269-330),
so a pixel's RNG position depends on the AO calls of all earlier pixels. The
one exchange step is therefore:

  1. each rank counts the AO calls of its rows           (backend.count)
  2. all_gather of the per-row counts (H x int32)         (RCCL over xGMI / gloo)
  3. every rank scans the full row vector in raster order -> its rows' RNG bases
  4. each rank shades its rows                            (backend.shade)
  5. gather of the int16 row tiles to rank 0, de-interleave

Backends: GpuRows (lib580rt.so through the C ABI, device tensors) and, for the
CPU tests of this logic with gloo, OracleRows in tests/.

render_frame() is the plain one-frame form. DistFrame is the steady-state form
over torch.distributed (any backend, the gloo CPU tests included): persistent
buffers, all_gather_into_tensor, the row-base scan as one kernel
(rt_gpu_row_bases), and a double-buffered asynchronous gather of frame N that
overlaps frame N+1's kernels. NativeRankFrame is bench.py's multi-rank step over
RCCL: the same exchange run by the library itself (rt_gpu_render_rank_async),
with the communicator and the frame loop native.
"""
import ctypes


def n_local_rows(height, rank, world):
    return len(range(rank, height, world))


def n_max_rows(height, world):
    return (height + world - 1) // world


class GpuRows:
    """Phase 1/2 of the C-ABI split (rt_gpu_count_rows / rt_gpu_shade_rows)."""

    def __init__(self, rt580, params, torch, device):
        self.rt580, self.lib, self.torch, self.device = rt580, rt580.load(), torch, device
        self.params = params
        self.width, self.height = params.width, params.height

    def _p(self, rank, world):
        p = self.rt580.RenderParams.from_buffer_copy(self.params)
        p.row_begin, p.row_end, p.row_step = rank, self.height, world
        return p

    def count(self, rank, world, persistent=False):
        """The per-row AO calls of this rank's rows (int32[n_max], padding rows
        0). persistent=True reuses one buffer per (rank, world) (DistFrame: the
        padding rows stay zero, the rows are rewritten every frame; its reader,
        the all-gather, is ordered before the next frame's count on the stream)."""
        t = self.torch
        if persistent:
            key = (rank, world)
            if getattr(self, "_cnt_key", None) != key:
                self._cnt = t.zeros(n_max_rows(self.height, world), dtype=t.int32, device=self.device)
                self._cnt_key = key
            out = self._cnt
        else:
            out = t.zeros(n_max_rows(self.height, world), dtype=t.int32, device=self.device)
        self._pc = self._p(rank, world)
        self.rt580.check(self.lib.rt_gpu_count_rows(ctypes.byref(self._pc), out.data_ptr()), "rt_gpu_count_rows")
        return out

    def shade(self, rank, world, local_base, out=None):
        t = self.torch
        fb = out if out is not None else \
            t.empty(n_max_rows(self.height, world) * self.width * 3, dtype=t.int16, device=self.device)
        self.rt580.check(self.lib.rt_gpu_shade_rows(ctypes.byref(self._pc), local_base.data_ptr(), fb.data_ptr()),
                         "rt_gpu_shade_rows")
        return fb

    def gamma_u8(self, fb, out):
        """FlushFrameBufferToPPM's pixel mapping on the device (rt_gpu_gamma_u8)."""
        self.rt580.check(self.lib.rt_gpu_gamma_u8(fb.data_ptr(), fb.numel(), out.data_ptr()), "rt_gpu_gamma_u8")
        return out

    def row_bases(self, gathered, rank, world, out):
        """gathered: int32[world * n_max] on the device -> out: int64[n_max] (one kernel)."""
        self.rt580.check(self.lib.rt_gpu_row_bases(gathered.data_ptr(), world, n_max_rows(self.height, world),
                                                   self.height, rank, out.data_ptr()), "rt_gpu_row_bases")
        return out


def render_frame(backend, dist, torch, height, width, rank, world, gather=True):
    """Render one frame across `world` ranks; returns the (H, W, 3) int16 frame
    on rank 0 (None elsewhere, or the local tile when gather=False)."""
    n_max = n_max_rows(height, world)
    counts = backend.count(rank, world)                       # int32[n_max], zero padded
    # gloo has no device collectives: stage through the host (tests / fallback
    # rehearsal of the multi-rank logic on one GPU); nccl (= RCCL) stays on device.
    stage = dist.get_backend() == "gloo" and counts.is_cuda
    dev = counts.device
    c_x = counts.cpu() if stage else counts
    gathered = [torch.empty_like(c_x) for _ in range(world)]
    dist.all_gather(gathered, c_x)
    if stage:
        gathered = [g.to(dev) for g in gathered]
    # row y lives on rank y % G at local index y // G
    full = torch.stack(gathered, dim=1).reshape(-1)[:height].to(torch.int64)
    base = torch.cumsum(full, 0) - full                       # exclusive scan, raster order
    local = base[rank::world]
    local_base = torch.zeros(n_max, dtype=torch.int64, device=counts.device)
    local_base[:local.numel()] = local
    fb = backend.shade(rank, world, local_base)               # int16[n_max*W*3]
    if not gather:
        return fb
    # int16 has no RCCL/gloo dtype: the tiles travel as their bytes
    fb_bytes = fb.view(torch.uint8)
    if stage:
        fb_bytes = fb_bytes.cpu()
    if rank == 0:
        tiles = [torch.empty_like(fb_bytes) for _ in range(world)]
        dist.gather(fb_bytes, gather_list=tiles, dst=0)
        if stage:
            tiles = [t.to(dev) for t in tiles]
        frame = torch.stack([t.view(torch.int16).view(n_max, width, 3) for t in tiles], dim=1)
        return frame.reshape(n_max * world, width, 3)[:height]
    dist.gather(fb_bytes, dst=0)
    return None


def render_frame_shared(backend, dist, torch, height, width, rank, world, body, lut):
    """The shared-body form of render_frame (what NativeRankFrame's library loop
    does with rt_gpu_rank_share_body, restated over torch.distributed for the
    gloo tests): each rank maps its rows to PPM bytes (`lut`, the writer's gamma
    table) and stores them at their places in `body` -- its view (H, W, 3) uint8
    of ONE frame shared by the ranks (SharedHostFrames) -- then a 4-byte
    all-gather says every rank's rows have landed. Returns body on rank 0."""
    import numpy as np
    fb = render_frame(backend, dist, torch, height, width, rank, world, gather=False)
    n = n_local_rows(height, rank, world)
    rows = fb.cpu().numpy().reshape(-1, width, 3)[:n]
    body[rank::world] = lut[np.clip(rows.astype(np.int64), 0, 255)]
    flag = torch.ones(1, dtype=torch.int32)
    dist.all_gather([torch.empty_like(flag) for _ in range(world)], flag)
    return body if rank == 0 else None


class DistFrame:
    """Steady-state multi-rank frames on the GPU backend over RCCL (see module doc).
    u8=True: each rank applies FlushFrameBufferToPPM's gamma mapping to its rows
    before the gather (3 B/px on the wire instead of 6), and rank 0
    writes the PPM body into registered host memory (rt_gpu_deinterleave_ppm);
    u8=False gathers the int16 Pixel framebuffer. The library's stream must be
    torch's current stream (rt_gpu_set_stream), which the collectives' waits
    order against."""

    def __init__(self, backend, dist, torch, height, width, rank, world, device, u8=True):
        self.b, self.dist, self.t = backend, dist, torch
        self.h, self.w, self.rank, self.world = height, width, rank, world
        self.u8 = u8
        self.n_max = n_max_rows(height, world)
        tile = self.n_max * width * 3
        self.gathered = torch.empty(world * self.n_max, dtype=torch.int32, device=device)
        self.base = torch.empty(self.n_max, dtype=torch.int64, device=device)
        self.fb = [torch.empty(tile, dtype=torch.int16, device=device) for _ in range(2)]
        self.fb8 = [torch.empty(tile, dtype=torch.uint8, device=device) for _ in range(2)] if u8 else None
        self.tiles = [torch.empty(world * tile * (1 if u8 else 2), dtype=torch.uint8, device=device)
                      for _ in range(2)] if rank == 0 else None
        self.frame = torch.empty(self.n_max * world, width, 3, dtype=torch.uint8 if u8 else torch.int16,
                                 device=device) if rank == 0 else None
        # rank 0: each assembled frame lands in page-locked host memory (a ring
        # of two, the frames in flight): a step ends with the frame on the
        # host, as the one-process paths' steps do. The u8 frame is
        # de-interleaved by the library straight into registered host buffers
        # (rt_gpu_deinterleave_ppm: one kernel writing through the host
        # mapping); the int16 frame is assembled by torch and copied.
        on_gpu = torch.device(device).type == "cuda"
        self.lib = getattr(backend, "lib", None) if (on_gpu and u8 and rank == 0) else None
        self.host = None
        self._reg = []
        if rank == 0 and on_gpu and self.lib is not None:
            import numpy as np
            span = (height * width * 3 + 4095) // 4096 * 4096
            for _ in range(2):
                raw = np.zeros(span + 4096, dtype=np.uint8)
                off = (-raw.ctypes.data) % 4096
                buf = raw[off:off + span]
                backend.rt580.check(self.lib.rt_gpu_host_register(buf.ctypes.data, span), "rt_gpu_host_register")
                self._reg.append((raw, buf))
            self.host = [torch.from_numpy(buf[:height * width * 3]).view(height, width, 3) for _, buf in self._reg]
            self.frame = None  # not used: the tiles go straight to the host buffers
        elif rank == 0 and on_gpu:
            self.host = [torch.empty(height, width, 3, dtype=self.frame.dtype, pin_memory=True) for _ in range(2)]
        self.host_i = 0
        self.last_host = None
        self.work = [None, None]
        self.i = 0
        self.pending = None  # buffer index whose gather is in flight and not yet de-interleaved

    def _assemble(self, k):
        if self.work[k] is not None:
            self.work[k].wait()  # stream-level: the compute stream waits for the collective
            self.work[k] = None
        if self.rank == 0:
            if self.lib is not None:  # u8 tiles -> the PPM body in registered host memory, one kernel
                self.last_host = self.host[self.host_i]
                self.b.rt580.check(self.lib.rt_gpu_deinterleave_ppm(
                    self.tiles[k].data_ptr(), self.world, self.n_max, self.w, self.h,
                    self._reg[self.host_i][1].ctypes.data, None), "rt_gpu_deinterleave_ppm")
                self.host_i ^= 1
                return
            tiles = (self.tiles[k] if self.u8 else self.tiles[k].view(self.t.int16)).view(
                self.world, self.n_max, self.w, 3)
            self.frame.view(self.n_max, self.world, self.w, 3).copy_(tiles.transpose(0, 1))
            if self.host is not None:
                self.last_host = self.host[self.host_i]
                self.last_host.copy_(self.frame[:self.h], non_blocking=True)
                self.host_i ^= 1

    def render(self):
        k = self.i
        if self.work[k] is not None:  # buffer k's gather (two frames ago) must be done before reuse
            self._assemble(k)
            self.pending = None
        counts = self.b.count(self.rank, self.world, persistent=True) if isinstance(self.b, GpuRows) else \
            self.b.count(self.rank, self.world)
        self.dist.all_gather_into_tensor(self.gathered, counts)
        self.b.row_bases(self.gathered, self.rank, self.world, self.base)
        fb = self.b.shade(self.rank, self.world, self.base, out=self.fb[k])
        if self.pending is not None:  # frame N-1: de-interleave now that frame N is queued
            self._assemble(self.pending)
        src = self.b.gamma_u8(fb, self.fb8[k]) if self.u8 else fb.view(self.t.uint8)
        if self.rank == 0:
            self.work[k] = self.dist.gather(src, gather_list=list(self.tiles[k].chunk(self.world)), dst=0,
                                            async_op=True)
        else:
            self.work[k] = self.dist.gather(src, dst=0, async_op=True)
        self.pending = k
        self.i ^= 1

    def finish(self):
        """Complete the last frame; returns the (H, W, 3) frame in rank 0's
        page-locked host memory (uint8 PPM pixels with u8=True, else the int16
        Pixel framebuffer), its copy complete."""
        if self.pending is not None:
            self._assemble(self.pending)
            self.pending = None
        for k in range(2):
            if self.work[k] is not None:
                self.work[k].wait()
                self.work[k] = None
        if self.rank != 0:
            return None
        if self.host is None:  # a CPU backend (gloo tests): the frame is host memory already
            return self.frame[:self.h]
        if self.lib is not None:
            self.b.rt580.check(self.lib.rt_gpu_synchronize(), "rt_gpu_synchronize")
        self.t.cuda.current_stream(self.tiles[0].device).synchronize()
        return self.last_host

    def close(self):
        """Complete what is in flight, then unregister rank 0's host buffers."""
        if self.pending is not None or any(w is not None for w in self.work):
            self.finish()
        for _, buf in self._reg:
            self.lib.rt_gpu_host_unregister(buf.ctypes.data)
        self._reg = []


def _broadcast_bytes(dist, data, nbytes, device, src=0):
    """`data` (bytes, on rank src) to every rank of `dist` as a uint8 tensor of
    nbytes (a device tensor unless the backend is gloo)."""
    import torch
    t = torch.zeros(nbytes, dtype=torch.uint8)
    if data is not None:
        t[:len(data)] = torch.tensor(list(data), dtype=torch.uint8)
    on_dev = dist.get_backend() != "gloo"
    u = t.to(device) if on_dev else t
    dist.broadcast(u, src=src)
    return bytes((u.cpu() if on_dev else u).tolist())


def _all_ranks(dist, ok, device):
    """True when every rank of `dist` passes ok = 1."""
    import torch
    t = torch.tensor([int(ok)], dtype=torch.int32)
    on_dev = dist.get_backend() != "gloo"
    u = t.to(device) if on_dev else t
    dist.all_reduce(u, op=dist.ReduceOp.MIN)
    return int(u.item()) == 1


class SharedHostFrames:
    """R frame bodies of `nbytes` each in ONE host mapping shared by the ranks
    of this node (NativeRankFrame's shared body): rank 0 creates a /dev/shm
    file and broadcasts its name over `dist`; every rank maps it; rank 0
    unlinks it once all have (the mappings stay until close)."""

    def __init__(self, dist, rank, nbytes, R, device=None):
        import mmap
        import os
        import secrets
        import numpy as np
        self.span = (nbytes + 4095) // 4096 * 4096
        size = self.span * R
        self.mm = None
        path = None
        if rank == 0:
            # the pages reserved now (a small tmpfs -- a container's 64 MB
            # /dev/shm -- fails here, not with SIGBUS at a write); "" = none
            path = "/dev/shm/rt580-%d-%s" % (os.getpid(), secrets.token_hex(6))
            try:
                fd = os.open(path, os.O_CREAT | os.O_EXCL | os.O_RDWR, 0o600)
                try:
                    os.posix_fallocate(fd, 0, size)
                except OSError:
                    os.close(fd)
                    os.unlink(path)
                    raise
            except OSError:
                path = ""
        name = _broadcast_bytes(dist, path.encode() if path is not None else None, 128,
                                device).rstrip(b"\0").decode()
        if not name:
            raise OSError("SharedHostFrames: no room for %d bytes in /dev/shm" % size)
        if rank != 0:
            fd = os.open(name, os.O_RDWR)
        try:
            self.mm = mmap.mmap(fd, size)
        finally:
            os.close(fd)
        dist.barrier()
        if rank == 0:
            os.unlink(name)
        self.arr = np.frombuffer(self.mm, dtype=np.uint8)
        self.bufs = [self.arr[k * self.span:(k + 1) * self.span] for k in range(R)]

    def close(self):
        self.bufs = []
        self.arr = None
        if self.mm is not None:
            try:
                self.mm.close()
            except BufferError:  # a caller still holds a view: the mapping goes with it
                pass
            self.mm = None


class NativeRankFrame:
    """The steady-state multi-rank frame driven by the library (bench.py's
    multi-rank step; rt_gpu_rank_* in include/rt580.h): the library owns the
    world's RCCL communicator (ncclCommInitRank from an id rank 0 makes and
    this class broadcasts over `dist`) and runs the rank's frame loop itself --
    count, all-gather, shading, the PPM bytes of its rows -- every collective on
    one library stream in the same order on every rank, two frames' AO phases
    overlapping. No per-frame Python, torch or event work beyond one ctypes call.

    shared (default): the ranks' PPM bodies are ONE host frame per ring entry,
    shared by the processes (SharedHostFrames; rt_gpu_rank_share_body): every
    rank writes its own rows into it over its own host link and a frame ends
    with a 4-byte all-gather. shared=False: rank 0 gathers the u8 row tiles over
    RCCL and writes the whole body (the form for ranks on different nodes).
    A ring of R host frames (frame k lands in buffer k mod R)."""

    R = 3
    ID_BYTES = 128  # NCCL_UNIQUE_ID_BYTES

    def __init__(self, rt580, params, dist, torch, height, width, rank, world, device, rehearse_gathered=None,
                 shared=True, host_frames=None):
        """rehearse_gathered (dist None): rank `rank` of `world` on this one GPU
        without a communicator, the world's per-row counts given (int32 device
        tensor [world * n_max]; rt580_rank_rehearse) -- one rank's share timed.
        host_frames: the R frame buffers (numpy uint8, page-aligned, >= H*W*3
        bytes) to write into instead of this class's own (a rehearsal's ranks
        run one after another into the same frames)."""
        import numpy as np
        self.rt580, self.lib, self.t = rt580, rt580.load(), torch
        self.params = rt580.RenderParams.from_buffer_copy(params)
        self.h, self.w, self.rank, self.world, self.shared = height, width, rank, world, shared
        if rehearse_gathered is not None:
            self._gathered = rehearse_gathered
            rt580.check(self.lib.rt580_rank_rehearse(world, rank, rehearse_gathered.data_ptr()), "rt580_rank_rehearse")
        else:
            uid = None
            if rank == 0:
                u = torch.zeros(self.ID_BYTES, dtype=torch.uint8)
                rt580.check(self.lib.rt_gpu_rank_unique_id(u.data_ptr(), self.ID_BYTES), "rt_gpu_rank_unique_id")
                uid = bytes(u.tolist())
            uid = _broadcast_bytes(dist, uid, self.ID_BYTES, device)
            ub = (ctypes.c_uint8 * self.ID_BYTES).from_buffer_copy(uid)
            rt580.check(self.lib.rt_gpu_rank_init(ctypes.addressof(ub), self.ID_BYTES, world, rank), "rt_gpu_rank_init")
        if shared:
            rt580.check(self.lib.rt_gpu_rank_share_body(1), "rt_gpu_rank_share_body")
        self._shm = None
        self._own = []  # private page-aligned buffers kept alive
        self._reg = []
        body = height * width * 3
        if host_frames is not None:
            self._register(list(host_frames))
        elif shared and world > 1 and dist is not None:
            # every rank maps and registers the shared ring, or (any failing)
            # all fall back to the gather form together: the two forms differ
            # in their collectives
            ok = 1
            try:
                self._shm = SharedHostFrames(dist, rank, body, self.R, device)
                self._register(self._shm.bufs)
            except (OSError, RuntimeError):
                ok = 0
            if not _all_ranks(dist, ok, device):
                self._unregister()
                if self._shm is not None:
                    self._shm.close()
                    self._shm = None
                rt580.check(self.lib.rt_gpu_rank_share_body(0), "rt_gpu_rank_share_body")
                self.shared = False
        if not self._reg and (self.shared or rank == 0):
            span = (body + 4095) // 4096 * 4096
            bufs = []
            for _ in range(self.R):
                raw = np.zeros(span + 4096, dtype=np.uint8)
                off = (-raw.ctypes.data) % 4096
                self._own.append(raw)
                bufs.append(raw[off:off + span])
            self._register(bufs)
        self.i = 0
        self.last = None

    def _register(self, bufs):
        for buf in bufs:
            self.rt580.check(self.lib.rt_gpu_host_register(buf.ctypes.data, buf.nbytes), "rt_gpu_host_register")
            self._reg.append(buf)

    def _unregister(self):
        for addr in [b.ctypes.data for b in self._reg]:
            self.lib.rt_gpu_host_unregister(addr)
        self._reg = []

    def render(self):
        host = self._reg[self.i].ctypes.data if self._reg else None
        self.rt580.check(self.lib.rt_gpu_render_rank_async(ctypes.byref(self.params), host),
                         "rt_gpu_render_rank_async")
        self.last = self.i
        self.i = (self.i + 1) % self.R

    def frame(self, k):
        """Rank 0: host buffer k of the ring as an (H, W, 3) uint8 array (after finish())."""
        return self._reg[k][:self.h * self.w * 3].reshape(self.h, self.w, 3)

    def finish(self):
        """Complete every frame in flight; rank 0: the last frame's PPM body
        (H, W, 3) uint8 in page-locked host memory."""
        self.rt580.check(self.lib.rt_gpu_rank_finish(), "rt_gpu_rank_finish")
        self.rt580.check(self.lib.rt_gpu_synchronize(), "rt_gpu_synchronize")
        if self.rank != 0 or self.last is None:
            return None
        return self.t.from_numpy(self.frame(self.last))

    def close(self):
        """The communicator and the host buffers (every frame complete first)."""
        self.lib.rt_gpu_rank_finish()
        self.lib.rt_gpu_synchronize()
        self.lib.rt_gpu_rank_shutdown()
        self._unregister()
        self._own = []
        if self._shm is not None:
            self._shm.close()
            self._shm = None
