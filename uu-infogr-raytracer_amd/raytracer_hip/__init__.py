"""raytracer_hip -- host-side mirror of the reference's plugin surface over libraytracer_hip.

Reference surface (Raytracer/RayTracer.cs, Raytracer/surface.cs):

    Surface(w, h)                  surface.cs:15-20   width, height, int[] pixels, Clear(c)
    RayTracer(Surface screen)      RayTracer.cs:535   .screen, Tick(), OnKeyPress(e), OnMouseMove(e)

Here `Surface.pixels` is a numpy int32 array (0x00RRGGBB, row-major y*width+x), and
`RayTracer.Tick()` renders the frame on the GPU through the C ABI (rt_render) straight into
it.  There is no CPU fallback: constructing a RayTracer without the built library or
without a gfx950 device raises RayTracerError.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi, debugview, scenes
from .abi import RayTracerError, check, load_library
from .debugview import SEGMENT_DTYPE, DebugView, surface_line, surface_print
from .dist import bands_of

__all__ = ["Surface", "RayTracer", "Context", "RayTracerError", "scenes", "abi", "load_library",
           "device_count", "camera_view", "wire_layout", "bands_of", "DebugView", "SEGMENT_DTYPE", "debugview"]


def device_count() -> int:
    lib = load_library()
    n = C.c_int(0)
    check(lib, lib.rt_device_count(C.byref(n)))
    return n.value


def wire_layout(width: int, height: int, band_rows: int, world: int, n_frames: int = 1) -> abi.rt_wire_layout:
    """rt_wire_layout_of: sizes of one rank's tile-codec wire (host only, no device needed)."""
    lib = load_library()
    out = abi.rt_wire_layout()
    check(lib, lib.rt_wire_layout_of(width, height, band_rows, world, n_frames, C.byref(out)))
    return out


def camera_view(camera: abi.rt_camera, width: int, height: int) -> abi.rt_view:
    lib = load_library()
    v = abi.rt_view()
    check(lib, lib.rt_camera_view(C.byref(camera), width, height, C.byref(v)))
    return v


class Surface:
    """surface.cs:7-46 -- the linear frame buffer the reference's Tick() fills."""

    def __init__(self, w: int, h: int):
        self.width = int(w)
        self.height = int(h)
        self.pixels = np.zeros(self.width * self.height, dtype=np.int32)

    def Clear(self, c: int):  # surface.cs:43-46
        self.pixels[:] = np.int32(c)

    def Line(self, x1: int, y1: int, x2: int, y2: int, c: int):  # surface.cs:57-100
        surface_line(self.pixels, self.width, self.height, x1, y1, x2, y2, c)

    def Print(self, t: str, x: int, y: int, c: int):  # surface.cs:107-131
        surface_print(self.pixels, self.width, t, x, y, c)

    def save_ppm(self, path: str):
        """Headless display hand-off (rt_write_ppm): the frame as a binary PPM."""
        lib = load_library()
        check(lib, lib.rt_write_ppm(path.encode(), self.pixels.ctypes.data, self.width, self.height))

    def image(self) -> np.ndarray:
        return self.pixels.reshape(self.height, self.width)


class Context:
    """Thin owner of an rt_ctx*."""

    def __init__(self, n_gpus: int = 1, flags: int = 0):
        """n_gpus band workers, one per device (rt_create_ex).  flags: abi.RT_CREATE_RCCL_GATHER routes
        rt_render through the RCCL gather to device 0 (even on one device); abi.RT_CREATE_SHARED_DEVICE
        puts every worker on the current device (the multi-GPU Tick rehearsed on one GPU)."""
        self.lib = load_library()
        self.ptr = C.c_void_p()
        check(self.lib, self.lib.rt_create_ex(int(n_gpus), int(flags), C.byref(self.ptr)))
        self.n_gpus = n_gpus
        self.scene = None

    # -- lifetime ---------------------------------------------------------------
    def close(self):
        if self.ptr:
            self.lib.rt_destroy(self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, code):
        return check(self.lib, code, self.ptr)

    # -- scene / camera -----------------------------------------------------------
    def set_scene(self, scene: scenes.Scene):
        S, P, L = scene.c_arrays()
        self._check(self.lib.rt_set_scene(self.ptr, S, len(scene.spheres), P, len(scene.planes), L,
                                          len(scene.lights), abi.rt_vec3(*scene.ambient), scene.recursion_limit))
        self._check(self.lib.rt_set_camera(self.ptr, C.byref(scene.c_camera())))
        self.scene = scene

    def set_camera(self, camera: abi.rt_camera):
        self._check(self.lib.rt_set_camera(self.ptr, C.byref(camera)))

    def set_view_height(self, view_height: int):
        """Later renders of a W x H frame trace rows [0, H) of a W x view_height view (0: H itself)."""
        self._check(self.lib.rt_set_view_height(self.ptr, int(view_height)))

    def set_counting(self, on: bool):
        """rt_set_counting (ABI 10): False = the trace launches count no rays (a display loop's setting; the
        pixels are the same), True = every launch adds its rays to stats() (the default)."""
        self._check(self.lib.rt_set_counting(self.ptr, 1 if on else 0))

    def get_camera(self) -> abi.rt_camera:
        c = abi.rt_camera()
        self._check(self.lib.rt_get_camera(self.ptr, C.byref(c)))
        return c

    # -- rendering ----------------------------------------------------------------
    def render(self, width: int, height: int, out: np.ndarray | None = None) -> np.ndarray:
        """Synchronous full frame into host memory (rt_render, the Tick() path)."""
        if out is None:
            out = np.empty(width * height, dtype=np.int32)
        assert out.dtype == np.int32 and out.flags.c_contiguous and out.size == width * height
        self._check(self.lib.rt_render(self.ptr, width, height, out.ctypes.data))
        return out.reshape(height, width)

    def render_device(self, width: int, height: int, d_ptr: int, stream: int = 0):
        self._check(self.lib.rt_render_device(self.ptr, width, height, C.c_void_p(d_ptr), C.c_void_p(stream)))

    def render_bands(self, width: int, height: int, band_rows: int, band_first: int, band_step: int, d_ptr: int,
                     stream: int = 0) -> int:
        nb = C.c_int(0)
        self._check(self.lib.rt_render_bands(self.ptr, width, height, band_rows, band_first, band_step,
                                             C.c_void_p(d_ptr), C.c_void_p(stream), C.byref(nb)))
        return nb.value

    def scatter_bands(self, width: int, height: int, band_rows: int, band_first: int, band_step: int,
                      d_bands: int, d_frame: int, stream: int = 0):
        self._check(self.lib.rt_scatter_bands(self.ptr, width, height, band_rows, band_first, band_step,
                                              C.c_void_p(d_bands), C.c_void_p(d_frame), C.c_void_p(stream)))

    def render_bands_ex(self, width: int, height: int, band_rows: int, band_first: int, band_step: int, d_ptr: int,
                        fmt: int = abi.RT_BANDS_RGB24, stream: int = 0) -> int:
        nb = C.c_int(0)
        self._check(self.lib.rt_render_bands_ex(self.ptr, width, height, band_rows, band_first, band_step,
                                                C.c_void_p(d_ptr), fmt, C.c_void_p(stream), C.byref(nb)))
        return nb.value

    def render_bands_batch(self, width: int, height: int, band_rows: int, band_first: int, band_step: int,
                           n_frames: int, d_ptr: int, frame_stride_bytes: int, fmt: int = abi.RT_BANDS_INT32,
                           stream: int = 0) -> int:
        """n_frames frames of these bands in one launch (rt_render_bands_batch)."""
        nb = C.c_int(0)
        self._check(self.lib.rt_render_bands_batch(self.ptr, width, height, band_rows, band_first, band_step, n_frames,
                                                   C.c_void_p(d_ptr), frame_stride_bytes, fmt, C.c_void_p(stream),
                                                   C.byref(nb)))
        return nb.value

    def scatter_gathered(self, width: int, height: int, band_rows: int, world: int, d_gathered: int,
                         rank_stride: int, d_frame: int, fmt: int = abi.RT_BANDS_RGB24, stream: int = 0):
        """Reassemble all ranks' band sets (rank r's at d_gathered + r * rank_stride) into d_frame."""
        self._check(self.lib.rt_scatter_gathered(self.ptr, width, height, band_rows, world, C.c_void_p(d_gathered),
                                                 rank_stride, fmt, C.c_void_p(d_frame), C.c_void_p(stream)))

    def encode_bands(self, width: int, height: int, band_rows: int, rank: int, world: int, d_bands: int,
                     frame_stride: int, n_frames: int, d_wire: int, d_wire_bytes: int = 0, stream: int = 0):
        """Tile-encode n_frames band sets of `rank` into the wire at d_wire (rt_encode_bands)."""
        self._check(self.lib.rt_encode_bands(self.ptr, width, height, band_rows, rank, world, C.c_void_p(d_bands),
                                             frame_stride, n_frames, C.c_void_p(d_wire),
                                             C.c_void_p(d_wire_bytes or None), C.c_void_p(stream)))

    def decode_gathered(self, width: int, height: int, band_rows: int, world: int, d_gathered: int,
                        rank_stride: int, n_frames: int, d_frames: int, frame_stride: int, stream: int = 0,
                        first_rank: int = 0):
        """Decode the wires of ranks first_rank.. (rank r's at d_gathered + r * rank_stride) into the frames."""
        self._check(self.lib.rt_decode_gathered(self.ptr, width, height, band_rows, world, first_rank,
                                                C.c_void_p(d_gathered),
                                                rank_stride, n_frames, C.c_void_p(d_frames), frame_stride,
                                                C.c_void_p(stream)))

    def render_bands_tiles(self, width: int, height: int, band_rows: int, rank: int, world: int, frame0: int,
                           n_frames: int, batch_frames: int, d_wire: int, stream: int = 0):
        """Frames frame0.. of a batch of `rank`'s bands traced straight into the wire's tile headers and
        the context's codec scratch (rt_render_bands_tiles; rt_finish_wire completes the wire)."""
        self._check(self.lib.rt_render_bands_tiles(self.ptr, width, height, band_rows, rank, world, frame0, n_frames,
                                                   batch_frames, C.c_void_p(d_wire), C.c_void_p(stream)))

    def finish_wire(self, width: int, height: int, band_rows: int, rank: int, world: int, n_frames: int,
                    d_wire: int, d_wire_bytes: int = 0, stream: int = 0):
        """The wire of the batch's first n_frames traced by render_bands_tiles (rt_finish_wire)."""
        self._check(self.lib.rt_finish_wire(self.ptr, width, height, band_rows, rank, world, n_frames,
                                            C.c_void_p(d_wire), C.c_void_p(d_wire_bytes or None), C.c_void_p(stream)))

    # -- one-process-per-GPU collectives on the caller's stream (rt_comm_*) --------------
    def comm_probe(self) -> bool:
        """True when RCCL can be loaded for rt_comm_* (rt_comm_probe; creates nothing)."""
        return self.lib.rt_comm_probe() == 0

    def comm_unique_id(self) -> bytes:
        """A new RCCL unique id (rank 0), to be shared with every rank (rt_comm_unique_id)."""
        buf = C.create_string_buffer(abi.RT_COMM_ID_BYTES)
        self._check(self.lib.rt_comm_unique_id(buf))
        return buf.raw

    def comm_init(self, world: int, rank: int, uid: bytes):
        """Join this context's device to a communicator of `world` ranks (collective; rt_comm_init)."""
        assert len(uid) == abi.RT_COMM_ID_BYTES
        self._check(self.lib.rt_comm_init(self.ptr, world, rank, C.create_string_buffer(uid, abi.RT_COMM_ID_BYTES)))

    def comm_allreduce_max_i64(self, d_ptr: int, count: int, stream: int = 0):
        self._check(self.lib.rt_comm_allreduce_max_i64(self.ptr, C.c_void_p(d_ptr), count, C.c_void_p(stream)))

    def comm_gather(self, d_send: int, n_bytes: int, d_recv: int, recv_stride: int, rotate: int = 0, stream: int = 0):
        """n_bytes of every rank's d_send to rank 0's d_recv slots ((r - rotate) mod world) * recv_stride."""
        self._check(self.lib.rt_comm_gather(self.ptr, C.c_void_p(d_send), n_bytes, C.c_void_p(d_recv or None),
                                            recv_stride, rotate, C.c_void_p(stream)))

    def render_async(self, width: int, height: int, out: np.ndarray):
        """Double-buffered Tick (rt_render_async): returns at once; `wait()` before reading `out`."""
        assert out.dtype == np.int32 and out.flags.c_contiguous and out.size == width * height
        self._check(self.lib.rt_render_async(self.ptr, width, height, out.ctypes.data))

    def wait(self):
        self._check(self.lib.rt_wait(self.ptr))

    def debug_segments(self, width: int, height: int, sample_stride: int = 0,
                       capacity: int = 0) -> tuple[np.ndarray, int]:
        """Visible-path segments of every `sample_stride`-th pixel (rt_debug_segments).
        Returns (segments, total appended); total > len(segments) means the buffer was full.
        sample_stride 0 picks one that samples about 4096 pixels."""
        if sample_stride <= 0:
            sample_stride = max(1, (width * height) // 4096)
        if capacity <= 0:
            n_pix = -(-(width * height) // sample_stride)
            capacity = n_pix * 8
        out = np.zeros(capacity, dtype=SEGMENT_DTYPE)
        n = C.c_int(0)
        self._check(self.lib.rt_debug_segments(self.ptr, width, height, sample_stride, out.ctypes.data,
                                               capacity, C.byref(n)))
        return out[:min(n.value, capacity)], n.value

    def register_host(self, arr: np.ndarray):
        self._check(self.lib.rt_register_host(self.ptr, C.c_void_p(arr.ctypes.data), arr.nbytes))

    def unregister_host(self, arr: np.ndarray):
        self._check(self.lib.rt_unregister_host(self.ptr, C.c_void_p(arr.ctypes.data)))

    # -- stats ----------------------------------------------------------------------
    def stats(self) -> dict:
        s = abi.rt_stats()
        self._check(self.lib.rt_get_stats(self.ptr, C.byref(s)))
        return s.as_dict()

    def reset_stats(self):
        self._check(self.lib.rt_reset_stats(self.ptr))

    def count_work(self, width: int, height: int) -> dict:
        """Nominal and executed work of one frame of the current camera (rt_count_work)."""
        w = abi.rt_work()
        self._check(self.lib.rt_count_work(self.ptr, width, height, C.byref(w)))
        return w.as_dict()

    def set_timing(self, every: int):
        """Time every `every`-th launch/copy/gather with HIP events (0 = none; default 64)."""
        self._check(self.lib.rt_set_timing(self.ptr, int(every)))

    def dispatch_order(self) -> int:
        """The single-frame dispatch order in use (0 rows by estimated cost, 1 rows bottom to top,
        2 rows varying fastest), -1 while the first launches still measure them (rt_dispatch_order)."""
        o = C.c_int(-1)
        self._check(self.lib.rt_dispatch_order(self.ptr, C.byref(o)))
        return o.value


class RayTracer:
    """RayTracer.cs:437-1062, public surface only, rendering on MI355X.

    `scene` defaults to the reference's hard-coded scene (RayTracer.cs:441-490).
    `debug=True` is the reference's DEBUG_ENABLE build: Tick() also composites the top-down
    ray inset (raytracer_hip.debugview) into the bottom-right corner of the frame.
    """

    _KEYS = {"W": abi.RT_KEY_W, "A": abi.RT_KEY_A, "S": abi.RT_KEY_S, "D": abi.RT_KEY_D,
             "Space": abi.RT_KEY_SPACE, "LeftShift": abi.RT_KEY_SHIFT, "RightShift": abi.RT_KEY_SHIFT}

    def __init__(self, screen: Surface, scene: scenes.Scene | None = None, n_gpus: int = 1,
                 debug: bool = False, debug_seed: int = 0):
        self.screen = screen
        self.debug = debug
        self._debug_seed = debug_seed
        self._ctx = Context(n_gpus)
        sc = scene or scenes.reference(screen.width, screen.height)
        self._scene = sc
        self._ctx.set_scene(sc)
        self._camera = sc.c_camera()
        self._ctx.register_host(screen.pixels)  # pin Surface.pixels once (D2H lands in it)

    def Tick(self):
        """RayTracer.Tick(), RayTracer.cs:886-935: the whole frame, synchronously."""
        self._ctx.set_camera(self._camera)
        self._ctx.render(self.screen.width, self.screen.height, self.screen.pixels)
        if self.debug:
            w, h = self.screen.width, self.screen.height
            segs, _ = self._ctx.debug_segments(w, h)
            DebugView(w, h).compose(self.screen.pixels, self._camera.position.tuple(), self._scene.spheres, segs,
                                    seed=self._debug_seed)
            self._debug_seed += 1

    def OnKeyPress(self, key):
        """RayTracer.OnKeyPress, RayTracer.cs:543-554 (key: 'W','A','S','D','Space','LeftShift'...)."""
        code = self._KEYS.get(key, 0) if isinstance(key, str) else int(key)
        check(self._ctx.lib, self._ctx.lib.rt_camera_on_key(C.byref(self._camera), code))

    def OnMouseMove(self, delta_x: float, delta_y: float):
        """RayTracer.OnMouseMove, RayTracer.cs:1058-1061."""
        check(self._ctx.lib, self._ctx.lib.rt_camera_on_mouse_move(C.byref(self._camera), delta_x, delta_y))

    @property
    def camera(self) -> abi.rt_camera:
        return self._camera

    def stats(self) -> dict:
        return self._ctx.stats()

    def close(self):
        if self._ctx.ptr:
            try:
                self._ctx.unregister_host(self.screen.pixels)
            finally:
                self._ctx.close()
