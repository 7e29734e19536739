"""Debug ray view host side: Surface.Line (surface.cs:51-100) and
the inset compositor (RayTracer.cs:878-954, :1022-1030).  CPU only; the GPU segment buffer
is covered in test_gpu_parity.py."""
import math

import numpy as np
import pytest

import raytracer_hip as rh
from raytracer_hip import abi
from raytracer_hip import debugview as dv


def _line_scalar(pixels, width, height, x1, y1, x2, y2, c):
    """Statement-by-statement scalar walk of surface.cs:57-100 (C# int semantics), the
    checker for the vectorised port."""
    def tdiv(a, b):
        q = abs(a) // abs(b)
        return q if (a >= 0) == (b >= 0) else -q

    def outcode(x, y):
        return (1 if x < 0 else (2 if x > width - 1 else 0)) + (4 if y < 0 else (8 if y > height - 1 else 0))

    xmin, ymin, xmax, ymax = 0, 0, width - 1, height - 1
    c0, c1 = outcode(x1, y1), outcode(x2, y2)
    accept = False
    while True:
        if c0 == 0 and c1 == 0:
            accept = True
            break
        if (c0 & c1) > 0:
            break
        co = c0 if c0 > 0 else c1
        x = y = 0
        if co & 8:
            x = x1 + tdiv((x2 - x1) * (ymax - y1), (y2 - y1)); y = ymax
        elif co & 4:
            x = x1 + tdiv((x2 - x1) * (ymin - y1), (y2 - y1)); y = ymin
        elif co & 2:
            y = y1 + tdiv((y2 - y1) * (xmax - x1), (x2 - x1)); x = xmax
        elif co & 1:
            y = y1 + tdiv((y2 - y1) * (xmin - x1), (x2 - x1)); x = xmin
        if co == c0:
            x1, y1 = x, y
            c0 = outcode(x1, y1)
        else:
            x2, y2 = x, y
            c1 = outcode(x2, y2)
    if not accept:
        return
    if abs(x2 - x1) >= abs(y2 - y1):
        if x2 < x1:
            x1, x2, y1, y2 = x2, x1, y2, y1
        n = x2 - x1
        if n == 0:
            return
        dy = tdiv((y2 - y1) * 8192, n)
        y1 *= 8192
        for _ in range(n):
            pixels[x1 + tdiv(y1, 8192) * width] = c
            x1 += 1
            y1 += dy
    else:
        if y2 < y1:
            x1, x2, y1, y2 = x2, x1, y2, y1
        n = y2 - y1
        if n == 0:
            return
        dx = tdiv((x2 - x1) * 8192, n)
        x1 *= 8192
        for _ in range(n):
            pixels[tdiv(x1, 8192) + y1 * width] = c
            y1 += 1
            x1 += dx


def test_line_known_answers():
    s = rh.Surface(8, 6)
    s.Line(1, 1, 5, 1, 7)  # horizontal: x = 1..4, end point not drawn
    assert s.image()[1].tolist() == [0, 7, 7, 7, 7, 0, 0, 0]
    s.Clear(0)
    s.Line(2, 5, 2, 0, 3)  # vertical, drawn from the lower y: rows 0..4
    assert s.image()[:, 2].tolist() == [3, 3, 3, 3, 3, 0]
    s.Clear(0)
    s.Line(0, 0, 4, 4, 1)  # diagonal
    assert [int(s.image()[i, i]) for i in range(5)] == [1, 1, 1, 1, 0]
    s.Clear(0)
    s.Line(3, 3, 3, 3, 9)  # zero length: nothing
    s.Line(-10, -1, -2, -5, 9)  # fully outside (shared outcode bit): nothing
    s.Line(20, 2, 30, 3, 9)
    assert not s.pixels.any()
    s.Line(-4, 2, 12, 2, 5)  # clipped to the window, the clipped end (x=7) not drawn
    assert s.image()[2].tolist() == [5] * 7 + [0]


def test_line_matches_scalar_walk_with_clipping():
    rng = np.random.default_rng(7)
    W, H = 37, 23
    a = np.zeros(W * H, dtype=np.int32)
    b = np.zeros(W * H, dtype=np.int32)
    for k in range(3000):
        x1, y1, x2, y2 = (int(v) for v in rng.integers(-60, 100, size=4))
        c = k + 1
        dv.surface_line(a, W, H, x1, y1, x2, y2, c)
        _line_scalar(b, W, H, x1, y1, x2, y2, c)
        assert np.array_equal(a, b), (k, x1, y1, x2, y2)


@pytest.mark.parametrize("w,h", [(640, 480), (1920, 1080), (97, 61), (3, 2)])
def test_debug_view_geometry(w, h):
    v = rh.DebugView(w, h)
    # DebugWidth/Height = (int)Math.Floor(w * 0.3f) (RayTracer.cs:878-879): float32 product
    assert v.debug_width == math.floor(float(np.float32(w) * np.float32(0.3)))
    assert v.debug_height == math.floor(float(np.float32(h) * np.float32(0.3)))
    m = v.inset_mask()
    assert m.sum() == max(0, w - v.top_left_x - 1) * max(0, h - v.top_left_y - 1)
    assert v.clamp((-5, 10**6)) == (v.top_left_x, h)


def test_offset_coordinates_known_answers():
    v = rh.DebugView(640, 480)
    assert (v.top_left_x, v.top_left_y) == (448, 336)
    # origin: (int)((320 + 0) * 0.3f) + 448, (int)((240 + 0 - 30) * 0.3f) + 336
    assert v.offset_coordinates((0.0, 0.0, 0.0)) == (544, 399)
    # z = 5: sy = -5 + 240, oy = 5 / 0.3f / 0.1f; (int)(371.666.. * 0.3f) = 111
    assert v.offset_coordinates((0.0, 3.0, 5.0)) == (544, 447)
    # NaN casts to int.MinValue (.NET x64), then wraps when offset
    x, y = v.offset_coordinates((float("nan"), 0.0, 0.0))
    assert x == dv._i32(-(1 << 31) + 448)


def test_kind_colours_are_shift_color_of_unit_rgb(oracle):
    assert dv.KIND_COLORS[dv.KIND_PRIMARY] == oracle.lib().oracle_shift_color(abi.rt_vec3(1.0, 0.0, 0.0))
    assert dv.KIND_COLORS[dv.KIND_SECONDARY] == oracle.lib().oracle_shift_color(abi.rt_vec3(0.0, 1.0, 0.0))
    assert dv.KIND_COLORS[dv.KIND_SHADOW] == oracle.lib().oracle_shift_color(abi.rt_vec3(0.0, 0.0, 1.0))
    assert dv.CIRCLE_COLOR == oracle.lib().oracle_shift_color(abi.rt_vec3(1.0, 1.0, 1.0))


def _synthetic_segments(n, seed=3):
    rng = np.random.default_rng(seed)
    seg = np.zeros(n, dtype=rh.SEGMENT_DTYPE)
    for f in ("ox", "oy", "oz", "ex", "ey", "ez"):
        seg[f] = rng.uniform(-12, 12, size=n).astype(np.float32)
    seg["kind"] = rng.integers(0, 3, size=n)
    seg["pixel"] = np.arange(n)
    return seg


def test_compose_draws_only_inside_inset_except_circles():
    W, H = 320, 240
    sc = rh.scenes.reference(W, H)
    frame = np.full(W * H, 0x123456, dtype=np.int32)
    v = rh.DebugView(W, H)
    out = v.compose(frame.copy(), (0.0, 0.0, 0.0), sc.spheres, _synthetic_segments(2000), seed=11)
    img = out.reshape(H, W)
    x0, y0 = v.top_left_x, v.top_left_y
    changed = img != 0x123456
    inside = np.zeros_like(changed)
    inside[y0:, x0:] = True  # lines are clamped to [TopLeft, width/height] then clipped
    assert (img[~inside][changed[~inside]] == dv.CIRCLE_COLOR).all()
    colours = set(np.unique(img[inside]).tolist())
    assert colours <= {0, 0x123456, *dv.KIND_COLORS.values(), dv.CIRCLE_COLOR}
    assert {0xFF0000, 0x00FF00, 0x0000FF} <= colours
    # deterministic for a seed, different picks for another
    again = v.compose(frame.copy(), (0.0, 0.0, 0.0), sc.spheres, _synthetic_segments(2000), seed=11)
    other = v.compose(frame.copy(), (0.0, 0.0, 0.0), sc.spheres, _synthetic_segments(2000), seed=12)
    assert np.array_equal(out, again) and not np.array_equal(out, other)


def test_compose_empty_pool_draws_circles_only():
    W, H = 160, 120
    sc = rh.scenes.reference(W, H)
    v = rh.DebugView(W, H)
    out = v.compose(np.zeros(W * H, dtype=np.int32), (0.0, 0.0, 0.0), sc.spheres,
                    np.zeros(0, dtype=rh.SEGMENT_DTYPE))
    assert set(np.unique(out).tolist()) <= {0, dv.CIRCLE_COLOR}
    assert (out == dv.CIRCLE_COLOR).any()
