"""FLAC metadata blocks and VORBIS_COMMENT tags: the mutagen.flac subset the reference uses.

The reference rewrites every encoded file with mutagen 1.47.0 (``converter.py:263-297``,
``spatial_encoder.py:309-375``): ``FLAC(path)``, ``.clear()``, ``f[KEY] = value`` in insertion
order, ``.save()``; and reads tags back with ``FLAC(path)[KEY][0]`` (``converter.py:329-379``,
``spatial_encoder.py:451-477``, ``cli.py:498-519``).  mutagen is not installed here, so the byte
layout it produces is restated (verified on ``test_data/sample_dem.flac``):

* blocks keep their order, PADDING blocks are dropped and ONE padding block is appended last;
* VORBIS_COMMENT keeps the vendor string; comments are ``KEY=value`` (key case as given, UTF-8),
  little-endian lengths, no framing bit;
* padding = ``available - needed`` when that is in ``[0, 10 KiB + 1 % of the audio]``, otherwise
  ``1024 + audio_bytes // 1000`` (``available`` = bytes of the old metadata blocks incl. their
  headers, ``needed`` = new non-padding blocks + the 4-byte padding header, audio = every byte
  after the old metadata, i.e. all later streams of a concatenated file).
"""

from __future__ import annotations

import struct
from pathlib import Path
from typing import Dict, Iterable, List, Optional, Sequence, Tuple, Union

STREAMINFO, PADDING, APPLICATION, SEEKTABLE, VORBIS_COMMENT, CUESHEET, PICTURE = 0, 1, 2, 3, 4, 5, 6


class FLACMetaError(ValueError):
    pass


def parse_blocks(data: bytes, at: int = 0) -> Tuple[List[Tuple[int, bytes]], int]:
    """``fLaC`` + metadata blocks at ``at`` -> ([(type, body)], first audio byte offset)."""
    if data[at:at + 4] != b"fLaC":
        raise FLACMetaError("not a FLAC stream (missing fLaC marker)")
    q = at + 4
    blocks = []
    while True:
        if q + 4 > len(data):
            raise FLACMetaError("truncated metadata block header")
        hdr = data[q]
        size = int.from_bytes(data[q + 1:q + 4], "big")
        body = data[q + 4:q + 4 + size]
        if len(body) != size:
            raise FLACMetaError("truncated metadata block")
        blocks.append((hdr & 0x7F, bytes(body)))
        q += 4 + size
        if hdr & 0x80:
            return blocks, q


def render_block(btype: int, body: bytes, last: bool) -> bytes:
    if len(body) >= 1 << 24:
        raise FLACMetaError("metadata block too large")
    return bytes([(0x80 if last else 0) | btype]) + len(body).to_bytes(3, "big") + body


class VorbisComment:
    """vendor + ordered ``(key, value)`` list with mutagen's case-insensitive dict view."""

    def __init__(self, vendor: str = "", comments: Optional[List[Tuple[str, str]]] = None):
        self.vendor = vendor
        self.comments: List[Tuple[str, str]] = list(comments or [])

    @classmethod
    def parse(cls, body: bytes) -> "VorbisComment":
        n = struct.unpack_from("<I", body, 0)[0]
        vendor = body[4:4 + n].decode("utf-8", "replace")
        q = 4 + n
        count = struct.unpack_from("<I", body, q)[0]
        q += 4
        out = []
        for _ in range(count):
            ln = struct.unpack_from("<I", body, q)[0]
            s = body[q + 4:q + 4 + ln].decode("utf-8", "replace")
            q += 4 + ln
            k, _, v = s.partition("=")
            out.append((k, v))
        return cls(vendor, out)

    def render(self) -> bytes:
        v = self.vendor.encode("utf-8")
        parts = [struct.pack("<I", len(v)), v, struct.pack("<I", len(self.comments))]
        for k, val in self.comments:
            if not k or any(c == "=" or not (0x20 <= ord(c) <= 0x7D) for c in k):
                raise FLACMetaError(f"invalid Vorbis comment key {k!r}")
            e = f"{k}={val}".encode("utf-8")
            parts += [struct.pack("<I", len(e)), e]
        return b"".join(parts)

    # mutagen VCommentDict view
    def __contains__(self, key: str) -> bool:
        k = key.lower()
        return any(c.lower() == k for c, _ in self.comments)

    def __getitem__(self, key: str) -> List[str]:
        k = key.lower()
        vals = [v for c, v in self.comments if c.lower() == k]
        if not vals:
            raise KeyError(key)
        return vals

    def get(self, key: str, default=None):
        try:
            return self[key]
        except KeyError:
            return default

    def __setitem__(self, key: str, value):
        k = key.lower()
        self.comments = [(c, v) for c, v in self.comments if c.lower() != k]
        for v in value if isinstance(value, list) else [value]:
            self.comments.append((key, v))

    def clear(self):
        self.comments = []

    def keys(self) -> List[str]:
        seen, out = set(), []
        for c, _ in self.comments:
            if c.lower() not in seen:
                seen.add(c.lower())
                out.append(c)
        return out


def default_padding(available_minus_needed: int, audio_bytes: int) -> int:
    """mutagen ``PaddingInfo._get_default_padding``."""
    high = 1024 * 10 + audio_bytes // 100
    low = 1024 + audio_bytes // 1000
    if available_minus_needed >= 0:
        return low if available_minus_needed > high else available_minus_needed
    return low


def rewrite_header_parts(header: bytes, audio_bytes: int, tags: Sequence[Tuple[str, str]], clear: bool = True) -> bytes:
    """The new metadata part (``fLaC`` + blocks + PADDING) of ``rewrite_header`` for a file whose metadata
    is ``header`` and whose audio is ``audio_bytes`` long (the audio itself is not needed)."""
    blocks, audio_off = parse_blocks(header, 0)
    kept: List[Tuple[int, bytes]] = []
    vc = None
    for bt, body in blocks:
        if bt == PADDING:
            continue
        if bt == VORBIS_COMMENT and vc is None:
            vc = VorbisComment.parse(body)
            kept.append((bt, b""))  # placeholder keeps the block position
        else:
            kept.append((bt, body))
    if vc is None:  # mutagen adds a VORBIS_COMMENT after STREAMINFO when the file has none
        vc = VorbisComment("")
        kept.insert(1, (VORBIS_COMMENT, b""))
    if clear:
        vc.clear()
    for k, v in tags:
        vc[k] = v
    out = bytearray()
    for bt, body in kept:
        out += render_block(bt, vc.render() if bt == VORBIS_COMMENT else body, False)
    available = audio_off - 4
    needed = len(out) + 4
    pad = max(default_padding(available - needed, audio_bytes), 0)
    out += render_block(PADDING, bytes(pad), True)
    return b"fLaC" + bytes(out)


def rewrite_header(data: bytes, tags: Sequence[Tuple[str, str]], clear: bool = True) -> bytes:
    """``FLAC(f); f.clear(); f[k] = v ...; f.save()`` on the bytes of a file -> new bytes."""
    _, audio_off = parse_blocks(data, 0)
    return rewrite_header_parts(data[:audio_off], len(data) - audio_off, tags, clear) + data[audio_off:]


class FLACFile:
    """Read-side tag access like ``mutagen.flac.FLAC(path)`` (tags as a case-insensitive dict)."""

    def __init__(self, src: Union[str, Path, bytes]):
        data = src if isinstance(src, (bytes, bytearray)) else Path(src).read_bytes()
        self.blocks, self.audio_offset = parse_blocks(bytes(data), 0)
        self.tags = VorbisComment("")
        for bt, body in self.blocks:
            if bt == VORBIS_COMMENT:
                self.tags = VorbisComment.parse(body)
                break
        si = next((b for t, b in self.blocks if t == STREAMINFO), None)
        if si is None or len(si) < 34:
            raise FLACMetaError("missing STREAMINFO")
        self.min_blocksize, self.max_blocksize = struct.unpack(">HH", si[:4])
        self.sample_rate = (si[10] << 12) | (si[11] << 4) | (si[12] >> 4)
        self.channels = ((si[12] >> 1) & 7) + 1
        self.bits_per_sample = (((si[12] & 1) << 4) | (si[13] >> 4)) + 1
        self.total_samples = ((si[13] & 15) << 32) | int.from_bytes(si[14:18], "big")

    def __contains__(self, key):
        return key in self.tags

    def __getitem__(self, key):
        return self.tags[key]

    def get(self, key, default=None):
        return self.tags.get(key, default)


def read_tags(src) -> Dict[str, str]:
    """First value of every tag, keys as stored."""
    vc = FLACFile(src).tags
    return {k: vc[k][0] for k in vc.keys()}


def embed_tags_file(path: Union[str, Path], tags: Iterable[Tuple[str, str]]):
    p = Path(path)
    p.write_bytes(rewrite_header(p.read_bytes(), list(tags)))
