"""Debug ray view and Surface.Line (rank 4).

The reference's only diagnostic is the `DEBUG_ENABLE` top-down inset (RayTracer.cs:2,
:423-435, :878-884, :903-954, :1022-1030): the bottom-right 30 % of the frame is left black,
the camera and every sphere are drawn as white circles, and 500 randomly picked traced rays
are drawn as lines coloured by RayKind (primary red, secondary green, shadow blue) with
Surface.Line (surface.cs:51-100).

Split here as: the GPU re-traces a strided sample of pixels and appends the segments of each
pixel's visible path to a device buffer (rt_debug_segments, debug_segments_kernel in
csrc/rt_kernel.hip); the host composites the inset with the functions below, which follow the
reference's integer/float arithmetic exactly (C# truncating division, float32 offsets,
(int) casts, OpenTK's float DegreesToRadians with double Math.Cos/Sin).

Documented differences from the reference (it is a diagnostic, not on the timed path):
  * the reference records every IntersectsSphere / IntersectPlane call (misses included,
    drawn as zero-length lines at the ray origin) into a ConcurrentBag through Task.Run, so
    its pool is dominated by misses and its order is nondeterministic; the GPU pool holds one
    segment per ray of each sampled pixel's visible path: the primary/secondary ray to its
    nearest hit (100 units long on a miss) and one shadow ray per light at diffuse hits,
    ending at the first blocking sphere in scene order (else at hitPoint + light.position,
    the reference's shadow-ray direction quirk, t = 1);
  * the 500 picks use a seeded numpy generator instead of an unseeded System.Random;
  * a circle point whose linear index falls outside the frame is skipped (the reference's
    SetPixel would throw IndexOutOfRangeException and end Tick).
"""
from __future__ import annotations

import math

import numpy as np

DEBUG_SIZE_SCALER = np.float32(0.3)  # RayTracer.cs:475
DEBUG_NUM_RAYS = 500                 # RayTracer.cs:917
KIND_PRIMARY, KIND_SECONDARY, KIND_SHADOW = 0, 1, 2
KIND_COLORS = {KIND_PRIMARY: 0xFF0000, KIND_SECONDARY: 0x00FF00, KIND_SHADOW: 0x0000FF}  # ShiftColor of unit RGB
CIRCLE_COLOR = 0xFFFFFF  # ShiftColor(VecUtil.FromFloat3(1))

SEGMENT_DTYPE = np.dtype([("ox", "<f4"), ("oy", "<f4"), ("oz", "<f4"), ("ex", "<f4"), ("ey", "<f4"),
                          ("ez", "<f4"), ("kind", "<i4"), ("pixel", "<i4")])

_F = np.float32
_INT_MIN = -(1 << 31)


def _i32(v: int) -> int:
    """C# unchecked int arithmetic (wrap to 32 bits)."""
    return ((int(v) + (1 << 31)) & 0xFFFFFFFF) - (1 << 31)


def _tdiv(a: int, b: int) -> int:
    """C# integer division (truncates toward zero)."""
    q = abs(a) // abs(b)
    return _i32(q if (a >= 0) == (b >= 0) else -q)


def _f2i(v) -> int:
    """.NET 6 x64 (int) cast of a float/double: truncation, INT_MIN for NaN/out of range."""
    v = float(v)
    if math.isnan(v) or not (-2147483649.0 < v < 2147483648.0):
        return _INT_MIN
    return int(v)


def _outcode(x: int, y: int, width: int, height: int) -> int:  # surface.cs:51-55
    xmax, ymax = width - 1, height - 1
    return (1 if x < 0 else (2 if x > xmax else 0)) + (4 if y < 0 else (8 if y > ymax else 0))


def surface_line(pixels: np.ndarray, width: int, height: int, x1: int, y1: int, x2: int, y2: int, c: int):
    """Surface.Line (surface.cs:57-100): Cohen-Sutherland clip to the window, then a 13-bit
    fixed-point DDA along the major axis writing l = |major delta| pixels (the end point is
    not drawn)."""
    xmin, ymin, xmax, ymax = 0, 0, width - 1, height - 1
    x1, y1, x2, y2 = _i32(x1), _i32(y1), _i32(x2), _i32(y2)
    c0, c1 = _outcode(x1, y1, width, height), _outcode(x2, y2, width, height)
    while True:
        if c0 == 0 and c1 == 0:
            break
        if c0 & c1:
            return
        x = y = 0
        co = c0 if c0 > 0 else c1
        if co & 8:
            x, y = _i32(x1 + _tdiv(_i32((x2 - x1) * (ymax - y1)), _i32(y2 - y1))), ymax
        elif co & 4:
            x, y = _i32(x1 + _tdiv(_i32((x2 - x1) * (ymin - y1)), _i32(y2 - y1))), ymin
        elif co & 2:
            y, x = _i32(y1 + _tdiv(_i32((y2 - y1) * (xmax - x1)), _i32(x2 - x1))), xmax
        elif co & 1:
            y, x = _i32(y1 + _tdiv(_i32((y2 - y1) * (xmin - x1)), _i32(x2 - x1))), xmin
        if co == c0:
            x1, y1 = x, y
            c0 = _outcode(x1, y1, width, height)
        else:
            x2, y2 = x, y
            c1 = _outcode(x2, y2, width, height)
    flat = pixels.reshape(-1)
    c = np.int32(_i32(c))
    # After clipping both ends are inside the window, so every fixed-point coordinate below
    # is non-negative and C#'s truncating "/ 8192" equals a floor.
    if abs(x2 - x1) >= abs(y2 - y1):
        if x2 < x1:
            x1, x2, y1, y2 = x2, x1, y2, y1
        n = x2 - x1
        if n == 0:
            return
        dy = _tdiv((y2 - y1) * 8192, n)
        i = np.arange(n, dtype=np.int64)
        flat[(x1 + i) + ((y1 * 8192 + i * dy) // 8192) * width] = c
    else:
        if y2 < y1:
            x1, x2, y1, y2 = x2, x1, y2, y1
        n = y2 - y1
        if n == 0:
            return
        dx = _tdiv((x2 - x1) * 8192, n)
        i = np.arange(n, dtype=np.int64)
        flat[(x1 * 8192 + i * dx) // 8192 + (y1 + i) * width] = c


class DebugView:
    """Geometry of the inset for a `width` x `height` screen (RayTracer.cs:878-884, :937-954)."""

    def __init__(self, width: int, height: int):
        self.width, self.height = int(width), int(height)
        self.debug_width = math.floor(float(_F(self.width) * DEBUG_SIZE_SCALER))
        self.debug_height = math.floor(float(_F(self.height) * DEBUG_SIZE_SCALER))
        self.top_left_x = self.width - self.debug_width
        self.top_left_y = self.height - self.debug_height

    def inset_mask(self) -> np.ndarray:
        """IsInDebugView(x, y): pixels TracePixel leaves unwritten (black after Clear(0))."""
        y, x = np.mgrid[0:self.height, 0:self.width]
        return (x > self.top_left_x) & (y > self.top_left_y)

    def offset_coordinates(self, p) -> tuple[int, int]:
        """DebugOffsetCoordinates (RayTracer.cs:944-954) of a world-space point (x, y, z)."""
        X, Z = _F(p[0]), _F(p[2])
        sx = (X + _F(self.width) / _F(2)) / _F(1)            # WorldspaceToScreenspace(.Xz)
        sy = (-Z + _F(self.height) / _F(2)) / _F(1)
        ox = X / DEBUG_SIZE_SCALER / _F(0.1)
        oy = Z / DEBUG_SIZE_SCALER / _F(0.1)
        with np.errstate(all="ignore"):
            cx = _f2i((sx + ox) * DEBUG_SIZE_SCALER)
            cy = _f2i((sy + oy - _F(30)) * DEBUG_SIZE_SCALER)
        return _i32(cx + self.top_left_x), _i32(cy + self.top_left_y)

    def clamp(self, q) -> tuple[int, int]:
        """ClampToDebugView (RayTracer.cs:937-942): Math.Clamp to [TopLeft, width/height]."""
        return (min(max(q[0], self.top_left_x), self.width), min(max(q[1], self.top_left_y), self.height))

    def draw_circle(self, pixels: np.ndarray, center, radius):
        """DrawCircle (RayTracer.cs:1022-1030): 360 points at whole degrees."""
        deg2rad = _F(math.pi) / _F(180)
        ang = np.arange(360, dtype=np.float32) * deg2rad
        r = float(_F(radius))
        with np.errstate(all="ignore"):
            fx = center[0] + r * np.cos(ang.astype(np.float64))
            fy = center[1] + r * np.sin(ang.astype(np.float64))
        flat = pixels.reshape(-1)
        for vx, vy in zip(fx, fy):
            idx = _i32(_i32(_f2i(vy) * self.width) + _f2i(vx))
            if 0 <= idx < flat.size:
                flat[idx] = np.int32(CIRCLE_COLOR)

    def compose(self, pixels: np.ndarray, camera_position, spheres, segments: np.ndarray,
                n_rays: int = DEBUG_NUM_RAYS, seed: int = 0):
        """The DEBUG_ENABLE part of Tick (RayTracer.cs:903-933) over a traced frame: black
        inset, camera and sphere circles, `n_rays` random segments as coloured lines."""
        img = pixels.reshape(self.height, self.width)
        img[self.inset_mask()] = 0
        self.draw_circle(pixels, self.offset_coordinates(camera_position), 1.0)
        for s in spheres:
            self.draw_circle(pixels, self.offset_coordinates(s.center),
                             _F(s.radius) / DEBUG_SIZE_SCALER / _F(0.5))
        if len(segments) == 0:
            return pixels
        picks = np.random.default_rng(seed).integers(0, len(segments), size=n_rays)
        for k in picks:
            g = segments[k]
            a = self.clamp(self.offset_coordinates((g["ox"], g["oy"], g["oz"])))
            b = self.clamp(self.offset_coordinates((g["ex"], g["ey"], g["ez"])))
            surface_line(pixels, self.width, self.height, a[0], a[1], b[0], b[1], KIND_COLORS[int(g["kind"])])
        return pixels
