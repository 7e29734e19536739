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


# -- Surface.Print (surface.cs:107-131) ---------------------------------------------------

def _print_scalar(pixels, width, t, x, y, c):
    """Statement-by-statement walk of surface.cs:121-130 over the atlas mask (C# IndexOutOfRange
    becomes IndexError at the first store outside the array)."""
    font = dv.font_mask().reshape(-1)
    fw = dv.font_mask().shape[1]
    fh = dv.font_mask().shape[0]
    redir = [0] * 256
    for i, ch in enumerate(dv.FONT_CHARS):
        redir[ord(ch) & 255] = i
    units = np.frombuffer(t.encode("utf-16-le"), dtype="<u2")
    for i, unit in enumerate(units):
        f = redir[int(unit) & 255]
        dest = x + i * 12 + y * width
        src = f * 12
        for v in range(fh):
            for u in range(12):
                if font[src + u]:
                    if not 0 <= dest + u < pixels.size:
                        raise IndexError(dest + u)
                    pixels[dest + u] = c
            src += fw
            dest += width


def test_font_mask_matches_the_reference_atlas():
    m = dv.font_mask()
    assert m.shape == (16, 1082)
    assert int(m.sum()) == 4676  # tools/make_font_mask.py over assets/font.png
    assert len(dv.FONT_CHARS) == 90 and 90 * dv.FONT_GLYPH_W <= m.shape[1]
    assert not m[:, 89 * 12:90 * 12].any()  # the space glyph is blank


@pytest.mark.parametrize("text,x,y", [("Hello, World!", 3, 2), ("0123456789 {}[];:<>,.?/\\", 0, 20),
                                      ("unknown: é€~|", 5, 40), ("", 0, 0),
                                      ("wraps into the next row", 150, 5)])
def test_print_matches_scalar_walk(text, x, y):
    W, H = 200, 64
    a = np.zeros(W * H, dtype=np.int32)
    b = a.copy()
    dv.surface_print(a, W, text, x, y, 0x123456)
    _print_scalar(b, W, text, x, y, 0x123456)
    np.testing.assert_array_equal(a, b)
    assert (a != 0).any() == any(ch != " " for ch in text)


def test_print_unknown_characters_use_glyph_zero():
    W, H = 40, 20
    a, b = np.zeros(W * H, dtype=np.int32), np.zeros(W * H, dtype=np.int32)
    dv.surface_print(a, W, "~", 1, 1, 7)   # '~' is not in the glyph table
    dv.surface_print(b, W, "A", 1, 1, 7)
    np.testing.assert_array_equal(a, b)
    s = rh.Surface(W, H)
    s.Print("A", 1, 1, 7)
    np.testing.assert_array_equal(s.pixels, b)


def test_print_out_of_range_raises_after_earlier_stores():
    W, H = 30, 20
    a, b = np.zeros(W * H, dtype=np.int32), np.zeros(W * H, dtype=np.int32)
    with pytest.raises(IndexError):
        dv.surface_print(a, W, "AB", 2, 10, 9)     # glyph rows run past the last row
    with pytest.raises(IndexError):
        _print_scalar(b, W, "AB", 2, 10, 9)
    np.testing.assert_array_equal(a, b)
    assert (a == 9).any()
    with pytest.raises(IndexError):
        dv.surface_print(np.zeros(W * H, dtype=np.int32), W, "A", -40, 0, 9)  # negative index
