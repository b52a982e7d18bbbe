"""Affine / Window / CRS: the three rasterio value types the encode path touches.

rasterio is not part of this image; the reference only uses these types as values
(``spatial_encoder.py:34-97``, ``cli.py:553-565``, ``converter.py:114-134``), so they are restated
here with rasterio's float evaluation order (the streaming index and tags are JSON renderings of
these numbers, so the rounding of every coordinate must match).
"""

from __future__ import annotations

from typing import Iterator, Optional, Tuple


class Affine(tuple):
    """``affine.Affine(a, b, c, d, e, f)``: x = a*col + b*row + c, y = d*col + e*row + f.

    ``list(Affine)`` has nine entries ``(a, b, c, d, e, f, 0, 0, 1)`` exactly like the affine
    package, which is what the reference serialises with ``list(src.transform)``.
    """

    def __new__(cls, a, b, c, d, e, f, g=0.0, h=0.0, i=1.0):
        return tuple.__new__(cls, (float(a), float(b), float(c), float(d), float(e), float(f), 0.0, 0.0, 1.0))

    a = property(lambda s: s[0])
    b = property(lambda s: s[1])
    c = property(lambda s: s[2])
    d = property(lambda s: s[3])
    e = property(lambda s: s[4])
    f = property(lambda s: s[5])

    @classmethod
    def identity(cls) -> "Affine":
        return cls(1.0, 0.0, 0.0, 0.0, 1.0, 0.0)

    @classmethod
    def translation(cls, x: float, y: float) -> "Affine":
        return cls(1.0, 0.0, x, 0.0, 1.0, y)

    def __mul__(self, other):
        sa, sb, sc, sd, se, sf = self[:6]
        if isinstance(other, Affine):
            oa, ob, oc, od, oe, of = other[:6]
            return Affine(sa * oa + sb * od, sa * ob + sb * oe, sa * oc + sb * of + sc,
                          sd * oa + se * od, sd * ob + se * oe, sd * oc + se * of + sf)
        vx, vy = other
        return (vx * sa + vy * sb + sc, vx * sd + vy * se + sf)

    def to_gdal(self) -> Tuple[float, ...]:
        return (self.c, self.a, self.b, self.f, self.d, self.e)

    def __repr__(self):
        return "Affine(%r, %r, %r,\n       %r, %r, %r)" % tuple(self[:6])


class Window:
    """``rasterio.windows.Window(col_off, row_off, width, height)``."""

    __slots__ = ("col_off", "row_off", "width", "height")

    def __init__(self, col_off: int, row_off: int, width: int, height: int):
        self.col_off, self.row_off, self.width, self.height = col_off, row_off, width, height

    def __iter__(self) -> Iterator[int]:
        return iter((self.col_off, self.row_off, self.width, self.height))

    def __eq__(self, other):
        return isinstance(other, Window) and tuple(self) == tuple(other)

    def __repr__(self):
        return f"Window(col_off={self.col_off}, row_off={self.row_off}, width={self.width}, height={self.height})"


def window_transform(transform: Affine, col_off: int, row_off: int) -> Affine:
    """``DatasetReader.window_transform(window)`` = ``rasterio.windows.transform``:
    ``Affine.translation(x - c, y - f) * transform`` with ``(x, y) = transform * (col, row)``."""
    x, y = transform * (float(col_off), float(row_off))
    return Affine.translation(x - transform.c, y - transform.f) * transform


def bounds(transform: Affine, width: int, height: int) -> Tuple[float, float, float, float]:
    """``DatasetReader.bounds`` -> (left, bottom, right, top) for a north-up transform."""
    a, b, c, d, e, f = transform[:6]
    if b == 0.0 and d == 0.0:
        return (c, f + e * height, c + a * width, f)
    xs = [c, c + a * width, c + b * height, c + a * width + b * height]
    ys = [f, f + d * width, f + e * height, f + d * width + e * height]
    return (min(xs), min(ys), max(xs), max(ys))


class CRS:
    """Holds the CRS string; ``str()``/``to_string()`` give ``"EPSG:n"`` like rasterio's CRS."""

    def __init__(self, s: Optional[str]):
        self._s = s or ""

    @classmethod
    def from_string(cls, s: str) -> "CRS":
        return cls(s)

    def to_string(self) -> str:
        return self._s

    def __str__(self):
        return self._s

    def __bool__(self):
        return bool(self._s)

    def __eq__(self, other):
        return str(self) == str(other)

    def __repr__(self):
        return f"CRS.from_string({self._s!r})"
