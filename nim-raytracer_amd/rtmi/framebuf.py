"""Framebuffer (src/utils/framebuf.nim) and colour transforms (src/utils/color.nim).

Layout is the ABI contract: w*h*3 float32, interleaved RGB, row-major, y = 0 is
the top row (framebuf.nim:10,19,25-28). Held here as a numpy array of shape
(h, w, 3) — the same bytes.
"""
import numpy as np


class Framebuf:
    def __init__(self, w, h):
        self.w = int(w)
        self.h = int(h)
        self.data = np.zeros((self.h, self.w, 3), dtype=np.float32)

    def __setitem__(self, xy, color):
        x, y = xy
        assert 0 <= x < self.w and 0 <= y < self.h
        self.data[y, x] = np.asarray(color, dtype=np.float64).astype(np.float32)

    def __getitem__(self, xy):
        x, y = xy
        assert 0 <= x < self.w and 0 <= y < self.h
        return self.data[y, x].copy()

    def rect(self, ox, oy, w, h, color):
        self.data[oy:oy + h, ox:ox + w] = np.asarray(color, dtype=np.float32)

    def writePpm(self, filename, bits=8, sRGB=True):
        return writePpm(self.data, filename, bits, sRGB)


def newFramebuf(w, h):
    return Framebuf(w, h)


def linearToSRGB(v):
    """color.nim:17-22 (vectorised)."""
    v = np.asarray(v, dtype=np.float64)
    a = 0.055
    return np.where(v <= 0.0031308, 12.92 * v, (1 + a) * np.power(np.maximum(v, 0.0), 1 / 2.4) - a)


def to_uint(data, bits=8, sRGB=True):
    """writePpm's outvalue (framebuf.nim:74-78): clamp (float32), sRGB
    (float64 inside, float32 result), round(c * maxval) as a float32 product
    rounded half away from zero (Nim round on float32). NaN -> 0."""
    maxval = np.float32(2 ** bits - 1)
    c = np.clip(np.nan_to_num(np.asarray(data, dtype=np.float32), nan=0.0), 0.0, 1.0).astype(np.float32)
    if sRGB:
        c = linearToSRGB(c.astype(np.float64)).astype(np.float32)
    x = c * maxval                      # float32 product
    r = np.floor(x)
    r = r + (x - r >= np.float32(0.5))  # half away from zero, exact in float32 (x >= 0)
    return r.astype(np.uint16 if bits > 8 else np.uint8)


def to_rgba(data, alpha=0xFF):
    """ImageRGBA.copyFrom (src/utils/image.nim:45-54): (h, w, 3) float32 ->
    (h, w, 4) uint8, round(c * 0xff) as a float32 product rounded half away
    from zero, no clamp; out-of-range results keep the low 8 bits of the
    x86-64 int32 conversion (NaN and |x| >= 2^31 -> INT32_MIN), as the
    reference's release build does (oracle_rgba_component)."""
    x = np.asarray(data, dtype=np.float32) * np.float32(255.0)
    with np.errstate(invalid="ignore"):
        a = np.abs(x)
        r = np.floor(a)
        r = r + (a - r >= np.float32(0.5))
        r = np.copysign(r, x)
        ok = (r >= -2147483648.0) & (r < 2147483648.0)
        i = np.where(ok, r, -2147483648.0).astype(np.int64)
    q = (i & 0xFF).astype(np.uint8)
    h, w = q.shape[0], q.shape[1]
    out = np.empty((h, w, 4), np.uint8)
    out[..., :3] = q
    out[..., 3] = alpha
    return out


def writePpm(data, filename, bits=8, sRGB=True):
    """P6 writer of framebuf.nim:55-93 (8-bit or big-endian 16-bit)."""
    data = np.asarray(data)
    h, w = data.shape[0], data.shape[1]
    q = to_uint(data.reshape(h, w, 3), bits, sRGB)
    maxval = 2 ** bits - 1
    try:
        with open(filename, "wb") as f:
            f.write(f"P6 {w} {h} {maxval} ".encode())
            f.write(q.astype(">u2").tobytes() if bits > 8 else q.tobytes())
        return True
    except OSError:
        return False
