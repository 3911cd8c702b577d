"""Minimal OpenEXR writer for loader tests (an independent encoder of the
OpenEXR 2 single-part layout: header attributes, offset table, scanline or
one-level tiled chunks; NONE / RLE / ZIPS / ZIP with the byte-interleave and
delta predictor of ImfZip/ImfRle). Used to check host/fs_image.cpp's LoadEXR
restatement against known pixel values."""
import struct
import zlib

import numpy as np

HALF, FLOAT, UINT = 1, 2, 0
NONE, RLE, ZIPS, ZIP, PIZ = 0, 1, 2, 3, 4


def _attr(name, typ, data):
    return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(data)) + data


def _predict_interleave(raw):
    """Inverse of the decoder's reorder + predictor."""
    b = np.frombuffer(raw, np.uint8)
    n = len(b)
    t = np.empty(n, np.uint8)
    half = (n + 1) // 2
    t[:half] = b[0::2]
    t[half:] = b[1::2]
    d = t.astype(np.int32)
    out = d.copy()
    out[1:] = (d[1:] - d[:-1] + 128) & 0xFF
    return out.astype(np.uint8).tobytes()


def _rle(data):
    out = bytearray()
    i, n = 0, len(data)
    while i < n:
        j = i + 1
        while j < n and data[j] == data[i] and j - i < 128:
            j += 1
        if j - i >= 3:
            out += struct.pack("b", j - i - 1) + bytes([data[i]])
            i = j
            continue
        j = i
        while j < n and j - i < 127:
            if j + 2 < n and data[j] == data[j + 1] == data[j + 2]:
                break
            j += 1
        j = max(j, i + 1)
        out += struct.pack("b", -(j - i)) + data[i:j]
        i = j
    return bytes(out)


def _compress(raw, comp):
    if comp == NONE:
        return raw
    pre = _predict_interleave(raw)
    c = zlib.compress(pre) if comp in (ZIP, ZIPS) else _rle(pre)
    return raw if len(c) >= len(raw) else c


def _lines_bytes(planes, types, rows, x0, x1):
    """Bytes of rows `rows` (per row: every channel's samples x0..x1)."""
    out = bytearray()
    for y in rows:
        for p, t in zip(planes, types):
            line = p[y, x0:x1]
            if t == HALF:
                out += line.astype("<f2").tobytes()
            elif t == FLOAT:
                out += line.astype("<f4").tobytes()
            else:
                out += line.astype("<u4").tobytes()
    return bytes(out)


def write(path, channels, compression=NONE, line_order=0, origin=(0, 0), tiles=None, flags=0):
    """channels: list of (name, pixel_type, HxW array) in file order."""
    names = [c[0] for c in channels]
    types = [c[1] for c in channels]
    planes = [np.asarray(c[2]) for c in channels]
    H, W = planes[0].shape
    x0, y0 = origin
    chl = b"".join(n.encode() + b"\0" + struct.pack("<iB3xii", t, 0, 1, 1) for n, t in zip(names, types)) + b"\0"
    hdr = _attr("channels", "chlist", chl)
    hdr += _attr("compression", "compression", bytes([compression]))
    box = struct.pack("<iiii", x0, y0, x0 + W - 1, y0 + H - 1)
    hdr += _attr("dataWindow", "box2i", box) + _attr("displayWindow", "box2i", box)
    hdr += _attr("lineOrder", "lineOrder", bytes([line_order]))
    hdr += _attr("pixelAspectRatio", "float", struct.pack("<f", 1.0))
    hdr += _attr("screenWindowCenter", "v2f", struct.pack("<ff", 0, 0))
    hdr += _attr("screenWindowWidth", "float", struct.pack("<f", 1.0))
    version = 2 | flags
    if tiles:
        hdr += _attr("tiles", "tiledesc", struct.pack("<IIB", tiles[0], tiles[1], 0))
        version |= 0x200
    head = struct.pack("<Ii", 20000630, version) + hdr + b"\0"
    chunks = []
    if not tiles:
        lines = 16 if compression == ZIP else (32 if compression == PIZ else 1)
        for b0 in range(0, H, lines):
            rows = range(b0, min(H, b0 + lines))
            data = _compress(_lines_bytes(planes, types, rows, 0, W), compression)
            chunks.append(struct.pack("<ii", y0 + b0, len(data)) + data)
    else:
        tx, ty = tiles
        for j in range(0, (H + ty - 1) // ty):
            for i in range(0, (W + tx - 1) // tx):
                rows = range(j * ty, min(H, (j + 1) * ty))
                data = _compress(_lines_bytes(planes, types, rows, i * tx, min(W, (i + 1) * tx)), compression)
                chunks.append(struct.pack("<iiiii", i, j, 0, 0, len(data)) + data)
    table_len = 8 * len(chunks)
    offs, pos, body = [], len(head) + table_len, b""
    for c in chunks:
        offs.append(pos)
        pos += len(c)
        body += c
    with open(path, "wb") as f:
        f.write(head + struct.pack(f"<{len(offs)}Q", *offs) + body)
