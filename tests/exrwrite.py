"""Minimal OpenEXR writer for loader tests (an independent encoder of the
OpenEXR 2 single-part layout: header attributes, offset table, scanline or
one-level tiled chunks; NONE / RLE / ZIPS / ZIP with the byte-interleave and
delta predictor of ImfZip/ImfRle; PIZ with the value bitmap and forward
lookup table, the 2D Haar wavelet (14-bit and modulo 16-bit bases) and the
run-length canonical Huffman coder of ImfPizCompressor/ImfHuf, written from
the format description with a plain heap Huffman code). Used to check
host/fs_image.cpp's LoadEXR restatement against known pixel values."""
import heapq
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


# ---- PIZ ------------------------------------------------------------------
def _wenc14(a, b):
    a = a - 65536 if a >= 32768 else a
    b = b - 65536 if b >= 32768 else b
    m, d = (a + b) >> 1, a - b
    return m & 0xFFFF, d & 0xFFFF


def _wenc16(a, b):
    ao = (a + 32768) & 0xFFFF
    m, d = (ao + b) >> 1, ao - b
    if d < 0:
        m = (m + 32768) & 0xFFFF
    return m, d & 0xFFFF


def _wav2_encode(buf, base, nx, ox, ny, oy, mx):
    """2D Haar transform in place of the layer buf[base + x*ox + y*oy],
    finest level first (the inverse of the decoder's loop)."""
    enc = _wenc14 if mx < (1 << 14) else _wenc16
    n = min(nx, ny)
    p, p2 = 1, 2
    while p2 <= n:
        y = 0
        while y <= ny - p2:
            x = 0
            while x <= nx - p2:
                i00 = base + y * oy + x * ox
                i01, i10 = i00 + p * ox, i00 + p * oy
                i11 = i10 + p * ox
                a00, a01 = enc(buf[i00], buf[i01])
                a10, a11 = enc(buf[i10], buf[i11])
                buf[i00], buf[i10] = enc(a00, a10)
                buf[i01], buf[i11] = enc(a01, a11)
                x += p2
            if nx & p:  # odd column
                i00 = base + y * oy + x * ox
                i10 = i00 + p * oy
                buf[i00], buf[i10] = enc(buf[i00], buf[i10])
            y += p2
        if ny & p:  # odd line
            x = 0
            while x <= nx - p2:
                i00 = base + y * oy + x * ox
                i01 = i00 + p * ox
                buf[i00], buf[i01] = enc(buf[i00], buf[i01])
                x += p2
        p, p2 = p2, p2 << 1


class _BitWriter:
    def __init__(self):
        self.out, self.c, self.lc = bytearray(), 0, 0

    def put(self, nbits, bits):
        self.c = (self.c << nbits) | bits
        self.lc += nbits
        while self.lc >= 8:
            self.lc -= 8
            self.out.append((self.c >> self.lc) & 0xFF)
        self.c &= (1 << self.lc) - 1

    def flush(self):
        nbits = len(self.out) * 8 + self.lc
        if self.lc:
            self.out.append((self.c << (8 - self.lc)) & 0xFF)
        return bytes(self.out), nbits


def _huf_compress(vals):
    """ImfHuf layout: im, iM, table length, bit count, 0; the code lengths
    of [im, iM] with zero runs; then the run-length coded symbols. iM is
    the run-length pseudo-symbol (largest value + 1)."""
    freq = {}
    for v in vals:
        freq[v] = freq.get(v, 0) + 1
    im, iM = min(freq), max(freq) + 1
    freq[iM] = 1
    # code lengths: a plain binary Huffman tree over the used symbols
    heap = [(f, i, (sym,)) for i, (sym, f) in enumerate(sorted(freq.items()))]
    heapq.heapify(heap)
    length = {sym: 0 for sym in freq}
    k = len(heap)
    while len(heap) > 1:
        f1, _, s1 = heapq.heappop(heap)
        f2, _, s2 = heapq.heappop(heap)
        for sym in s1 + s2:
            length[sym] += 1
        heapq.heappush(heap, (f1 + f2, k, s1 + s2))
        k += 1
    assert max(length.values()) <= 58
    # canonical codes: per length, codes ascend with the symbol; shorter
    # codes are numerically higher (padded with zeroes on the right)
    count = [0] * 59
    for sym in length:
        count[length[sym]] += 1
    count[0] += 65537 - len(length)
    first, c = [0] * 59, 0
    for ln in range(58, 0, -1):
        first[ln], c = c, (c + count[ln]) >> 1
    code = {}
    for sym in sorted(length):
        ln = length[sym]
        code[sym] = (first[ln], ln)
        first[ln] += 1
    # the packed length table (zero runs: 59..62 short, 63 + 8 bits long)
    tw = _BitWriter()
    i = im
    while i <= iM:
        ln = length.get(i, 0)
        if ln == 0:
            run = 1
            while i < iM and run < 255 + 6 and length.get(i + 1, 0) == 0:
                i += 1
                run += 1
            if run >= 2:
                if run >= 6:
                    tw.put(6, 63)
                    tw.put(8, run - 6)
                else:
                    tw.put(6, 59 + run - 2)
                i += 1
                continue
        tw.put(6, ln)
        i += 1
    table, _ = tw.flush()
    dw = _BitWriter()

    def send(sym, run):
        cs, ls = code[sym]
        cr, lr = code[iM]
        if ls + lr + 8 < ls * run:
            dw.put(ls, cs)
            dw.put(lr, cr)
            dw.put(8, run)
        else:
            for _ in range(run + 1):
                dw.put(ls, cs)

    s, run = vals[0], 0
    for v in vals[1:]:
        if v == s and run < 255:
            run += 1
        else:
            send(s, run)
            run = 0
        s = v
    send(s, run)
    data, nbits = dw.flush()
    return struct.pack("<IIIII", im, iM, len(table), nbits, 0) + table + data


def _piz(raw, types, width, nlines):
    """One PIZ block of `nlines` lines (each line: every channel's samples)."""
    words = np.frombuffer(raw, "<u2")
    sizes = [1 if t == HALF else 2 for t in types]
    # channel-major layers buffer: per channel its rows of width*size words
    chan = []
    pos = 0
    rows = [[] for _ in types]
    for _ in range(nlines):
        for c, sz in enumerate(sizes):
            rows[c].append(words[pos:pos + width * sz])
            pos += width * sz
    for c in range(len(types)):
        chan.append(np.concatenate(rows[c]) if rows[c] else np.zeros(0, np.uint16))
    buf = np.concatenate(chan).astype(np.int64)
    present = np.zeros(65536, bool)
    present[buf] = True
    present[0] = True
    bitmap = np.packbits(present, bitorder="little")
    bitmap[0] &= 0xFE  # zero is implied
    nz = np.nonzero(bitmap)[0]
    lo, hi = (int(nz[0]), int(nz[-1])) if len(nz) else (8191, 0)
    fwd = np.cumsum(present) - 1
    max_value = int(fwd[-1])
    vals = [int(v) for v in fwd[buf]]
    base = 0
    for c, sz in enumerate(sizes):
        for j in range(sz):
            _wav2_encode(vals, base + j, width, sz, nlines, width * sz, max_value)
        base += width * nlines * sz
    out = struct.pack("<HH", lo, hi)
    if lo <= hi:
        out += bitmap[lo:hi + 1].tobytes()
    huf = _huf_compress(vals)
    return out + struct.pack("<i", len(huf)) + huf


def _compress(raw, comp, types=None, width=0, nlines=0):
    if comp == NONE:
        return raw
    if comp == PIZ:
        c = _piz(raw, types, width, nlines)
        return raw if len(c) >= len(raw) else c
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
            data = _compress(_lines_bytes(planes, types, rows, 0, W), compression, types, W, len(rows))
            chunks.append(struct.pack("<ii", y0 + b0, len(data)) + data)
    else:
        tx, ty = tiles
        for j in range(0, (H + ty - 1) // ty):
            for i in range(0, (W + tx - 1) // tx):
                rows = range(j * ty, min(H, (j + 1) * ty))
                x1 = min(W, (i + 1) * tx)
                data = _compress(_lines_bytes(planes, types, rows, i * tx, x1), compression, types, x1 - i * tx,
                                 len(rows))
                chunks.append(struct.pack("<iiiii", i, j, 0, 0, len(data)) + data)
    table_len = 8 * len(chunks)
    offs, pos, body = [], len(head) + table_len, b""
    for c in chunks:
        offs.append(pos)
        pos += len(c)
        body += c
    with open(path, "wb") as f:
        f.write(head + struct.pack(f"<{len(offs)}Q", *offs) + body)
