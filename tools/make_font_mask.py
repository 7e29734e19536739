"""Generate raytracer_hip/data/font_mask.bin from the reference's font atlas (run here, where
/root/reference exists; the output is committed).

Surface.Print (Raytracer/surface.cs:107-131) loads assets/font.png through the file ctor
(:22-31, ImageSharp Bgra32) and only ever tests `(pixel & 0xffffff) != 0`, i.e. whether any
of R, G, B is nonzero.  So the atlas is kept as that bit mask:
    u16 width, u16 height (little endian), then np.packbits(mask[height][width]) row-major.
"""
import struct
import sys
from pathlib import Path

import numpy as np
from PIL import Image

src = Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/Raytracer/assets/font.png")
dst = Path(__file__).resolve().parents[1] / "uu-infogr-raytracer_amd/raytracer_hip/data/font_mask.bin"
rgb = np.asarray(Image.open(src).convert("RGB"))
mask = rgb.any(axis=2)
h, w = mask.shape
dst.write_bytes(struct.pack("<HH", w, h) + np.packbits(mask.reshape(-1)).tobytes())
print(f"{dst}: {w}x{h}, {int(mask.sum())} set pixels")
