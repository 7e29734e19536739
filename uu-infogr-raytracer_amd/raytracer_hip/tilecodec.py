"""Lossless tile codec for shipping band sets to rank 0 -- host mirror.

The multi-GPU frame is gathered to rank 0 over xGMI every frame; at 1080p that transfer, not
the trace, bounds strong scaling.  Rendered frames are mostly flat (sky,
checkerboard tiles, slowly varying shading at 8 bits per channel), so each rank encodes its
band sets before the gather and rank 0 decodes them straight into the frame:

* A band set (this rank's bands packed one after the other, `RowBands`) is cut into 8x8
  tiles over its local rows: tile (tr, tc) = local rows 8tr..8tr+7, columns 8tc..8tc+7.
  Every rank uses the tile grid of the largest band set (`max_bands` bands), so the fixed
  part of the wire has the same size on every rank.  A batch of F frames is F tile grids
  one after the other.
* Pixel (rx, ry) of a tile is predicted by its left neighbour; the first column by the pixel
  above in odd rows and by the tile's first pixel in even rows (on the GPU a lane holds one
  tile row: the left prediction runs in registers, the row above is one DPP row shift, the
  first pixel one broadcast); pixel (0, 0) is stored raw in the tile header.  Residuals
  are per channel, modulo 256, zigzag-mapped to 0..255 (0, -1, 1, -2, ... -> 0, 1, 2, 3).
  Pixels outside the frame (columns >= width, rows of missing bands or past the height)
  have residual 0 and are never written by the decoder.
* Channel c (R, G, B) of a tile gets a width w_c in {0, 1, 2, 4, 8}: the bit length of its
  largest zigzag residual rounded up to a power of two.  Its segment is w_c 8-byte units =
  64 * w_c bits, lane l's residual at bits [l*w_c, (l+1)*w_c) of the little-endian stream
  (inside one 32-bit word, since w_c divides 32): a tile row's residuals of a channel are
  w_c consecutive bytes, one store / load per GPU lane.
* Tiles are grouped in chunks of 8 consecutive tiles (one wave's tiles on the GPU); a
  tile's payload offset is its chunk's base (a 32-bit unit offset, one per chunk) plus its
  offset inside the chunk (kept in the header).  Segments follow each other R, G, B.

Wire layout of one rank's batch (little endian; `layout()` gives the sizes):
    [0:16)                 u32 total_units, n_tiles, n_chunks, tiles_per_frame
    [16 : 16+8T)           per tile: u32 first pixel 0x00RRGGBB,
                                     u32 meta = w_R | w_G << 4 | w_B << 8 | rel_offset << 12
    [.. : +4*NC)           u32 chunk base (units), then padding to 8 bytes = fixed_bytes
    [fixed_bytes : +8*total_units)   payload units, tile after tile, segments R, G, B
The encoding is deterministic: the GPU encoder (rt_encode_bands) produces exactly these
bytes, and rt_decode_gathered reproduces the band pixels bit for bit.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .dist import bands_of

TILE = 8
_L = np.arange(64)
# predictor lane of every lane: left; first column: above (odd rows) or lane 0 (even rows)
PRED_SRC = np.where(_L % 8 > 0, _L - 1, np.where((_L // 8) % 2 == 1, _L - 8, 0))
CHUNK = 8
HEADER_BYTES = 16
MAX_UNITS_PER_TILE = 24


@dataclass(frozen=True)
class WireLayout:
    tiles_x: int
    tiles_y: int
    tiles_per_frame: int
    n_frames: int
    n_tiles: int
    n_chunks: int
    fixed_bytes: int
    max_bytes: int  # fixed part + the largest possible payload

    def wire_bytes(self, total_units: int) -> int:
        return self.fixed_bytes + 8 * int(total_units)


def layout(width: int, height: int, band_rows: int, world: int, n_frames: int = 1) -> WireLayout:
    """Sizes of one rank's wire (the same for every rank of `world`)."""
    if width <= 0 or height <= 0 or band_rows <= 0 or world <= 0 or n_frames <= 0:
        raise ValueError("bad wire layout arguments")
    rows = max(1, bands_of(height, band_rows, 0, world)) * band_rows
    tx, ty = -(-width // TILE), -(-rows // TILE)
    tpf = tx * ty
    nt = tpf * n_frames
    nc = -(-nt // CHUNK)
    fixed = HEADER_BYTES + 8 * nt + 4 * nc
    fixed = (fixed + 7) // 8 * 8
    return WireLayout(tx, ty, tpf, n_frames, nt, nc, fixed, fixed + 8 * MAX_UNITS_PER_TILE * nt)


def _valid_mask(width, height, band_rows, rank, world, lay):
    """[ty*8, tx*8] bool: pixel of the band set that exists in the frame."""
    rows, cols = lay.tiles_y * TILE, lay.tiles_x * TILE
    nb = bands_of(height, band_rows, rank, world)
    r = np.arange(rows)
    y = (rank + (r // band_rows) * world) * band_rows + r % band_rows
    row_ok = (r < nb * band_rows) & (y < height)
    col_ok = np.arange(cols) < width
    return row_ok[:, None] & col_ok[None, :]


def _tiles(img, lay):
    """[F, rows, cols] -> [F*T, 64] lanes (tile-major, lane = ry*8 + rx)."""
    F = img.shape[0]
    t = img.reshape(F, lay.tiles_y, TILE, lay.tiles_x, TILE).transpose(0, 1, 3, 2, 4)
    return t.reshape(F * lay.tiles_per_frame, TILE * TILE)


def encode(bands, width: int, height: int, band_rows: int, rank: int, world: int, n_frames: int = 1) -> bytes:
    """Encode n_frames band sets of `rank` (int32 0x00RRGGBB, each max_bands*band_rows x width,
    frame after frame; anything at invalid pixels is ignored) into the wire bytes."""
    lay = layout(width, height, band_rows, world, n_frames)
    slot_rows = max(1, bands_of(height, band_rows, 0, world)) * band_rows
    img = np.asarray(bands, dtype=np.int32).reshape(n_frames, slot_rows, width)
    rows, cols = lay.tiles_y * TILE, lay.tiles_x * TILE
    pad = np.zeros((n_frames, rows, cols), dtype=np.int64)
    pad[:, :slot_rows, :width] = img.astype(np.int64) & 0xFFFFFF
    valid = np.broadcast_to(_valid_mask(width, height, band_rows, rank, world, lay), pad.shape)
    v = _tiles(pad, lay)
    ok = _tiles(np.ascontiguousarray(valid), lay)
    lane = np.arange(64)
    rx, ry = lane % 8, lane // 8
    src = PRED_SRC
    pred = v[:, src]
    ch = np.stack([(v >> s) & 255 for s in (16, 8, 0)], -1)        # [T, 64, 3] R, G, B
    pch = np.stack([(pred >> s) & 255 for s in (16, 8, 0)], -1)
    d = (ch - pch) & 255
    d[:, 0, :] = 0
    d[~ok] = 0
    s8 = np.where(d >= 128, d - 256, d)
    z = np.where(s8 >= 0, 2 * s8, -2 * s8 - 1).astype(np.int64)    # [T, 64, 3]
    orz = np.bitwise_or.reduce(z, axis=1)                           # [T, 3]
    w = np.zeros_like(orz)
    for k in range(8):                                              # bit length ...
        w = np.where(orz >> k != 0, k + 1, w)
    w = np.select([w == 0, w == 1, w == 2, w <= 4], [0, 1, 2, 4], 8)  # ... rounded up to 0/1/2/4/8
    units = w.sum(axis=1)
    nt, nc = lay.n_tiles, lay.n_chunks
    units_pad = np.zeros(nc * CHUNK, dtype=np.int64)
    units_pad[:nt] = units
    per_chunk = units_pad.reshape(nc, CHUNK)
    rel = (np.cumsum(per_chunk, axis=1) - per_chunk).reshape(-1)[:nt]
    chunk_tot = per_chunk.sum(axis=1)
    chunk_base = np.cumsum(chunk_tot) - chunk_tot
    total = int(chunk_tot.sum())
    first = np.where(ok[:, 0], v[:, 0], 0)
    meta = w[:, 0] | (w[:, 1] << 4) | (w[:, 2] << 8) | (rel << 12)
    out = bytearray(lay.wire_bytes(total))
    hdr = np.array([total, nt, nc, lay.tiles_per_frame], dtype=np.uint32)
    out[0:16] = hdr.tobytes()
    th = np.stack([first, meta], -1).astype(np.uint32)
    out[16:16 + 8 * nt] = th.tobytes()
    out[16 + 8 * nt:16 + 8 * nt + 4 * nc] = chunk_base.astype(np.uint32).tobytes()
    # payload: segments of tile t at chunk_base[t // CHUNK] + rel[t], R then G then B
    words = np.zeros(2 * total, dtype=np.uint64)  # u32 words (kept in u64 for the shifts)
    base = chunk_base[np.arange(nt) // CHUNK] + rel
    for t in np.nonzero(units)[0]:
        o = 2 * int(base[t])
        for c in range(3):
            wc = int(w[t, c])
            if wc:
                pos = lane * wc
                np.bitwise_or.at(words, o + (pos >> 5), (z[t, :, c].astype(np.uint64) << (pos & 31).astype(np.uint64)))
                o += 2 * wc
    planes = words.astype(np.uint32)
    out[lay.fixed_bytes:] = planes.tobytes()
    return bytes(out)


def decode_into(frames, wire, width: int, height: int, band_rows: int, rank: int, world: int) -> int:
    """Decode one rank's wire into frames [F, height, width] (int32, written in place at the
    rank's pixels only).  Returns the number of payload units read."""
    wire = np.frombuffer(bytes(wire), dtype=np.uint8)
    total, nt, nc, tpf = (int(x) for x in wire[:16].view(np.uint32))
    F = nt // tpf
    lay = layout(width, height, band_rows, world, F)
    if (nt, nc, tpf) != (lay.n_tiles, lay.n_chunks, lay.tiles_per_frame):
        raise ValueError("wire does not match the layout")
    th = wire[16:16 + 8 * nt].view(np.uint32).reshape(nt, 2).astype(np.int64)
    chunk_base = wire[16 + 8 * nt:16 + 8 * nt + 4 * nc].view(np.uint32).astype(np.int64)
    words = wire[lay.fixed_bytes:lay.fixed_bytes + 8 * total].view(np.uint32).astype(np.int64)
    first, meta = th[:, 0], th[:, 1]
    w = np.stack([(meta >> s) & 15 for s in (0, 4, 8)], -1)
    rel = meta >> 12
    base = chunk_base[np.arange(nt) // CHUNK] + rel
    lane = np.arange(64)
    z = np.zeros((nt, 64, 3), dtype=np.int64)
    for t in np.nonzero(w.sum(axis=1))[0]:
        o = 2 * int(base[t])
        for c in range(3):
            wc = int(w[t, c])
            if wc:
                pos = lane * wc
                z[t, :, c] = (words[o + (pos >> 5)] >> (pos & 31)) & ((1 << wc) - 1)
                o += 2 * wc
    d = ((z >> 1) ^ -(z & 1)) & 255                                 # [T, 64, 3]
    val = np.zeros_like(d)
    val[:, 0] = np.stack([(first >> s) & 255 for s in (16, 8, 0)], -1)
    for ln in range(1, 64):                                         # predictors precede their lane
        val[:, ln] = (val[:, PRED_SRC[ln]] + d[:, ln]) & 255
    val = val.reshape(nt, 8, 8, 3)                                  # [T, ry, rx, c]
    px = (val[..., 0] << 16) | (val[..., 1] << 8) | val[..., 2]     # [T, ry, rx]
    img = px.reshape(F, lay.tiles_y, lay.tiles_x, 8, 8).transpose(0, 1, 3, 2, 4)
    img = img.reshape(F, lay.tiles_y * 8, lay.tiles_x * 8)
    valid = _valid_mask(width, height, band_rows, rank, world, lay)
    r_idx, x_idx = np.nonzero(valid)
    y_idx = (rank + (r_idx // band_rows) * world) * band_rows + r_idx % band_rows
    fr = np.asarray(frames).reshape(F, height, width)
    fr[:, y_idx, x_idx] = img[:, r_idx, x_idx].astype(np.int32)
    return total
