"""TEST INFRASTRUCTURE ONLY (the checker, never the product): an independent numpy restatement of
the JPEG decoding the reference performs with stb_image 2.06 (stbi_load(file, &w, &h, &comp, 0),
path_tracer/src/sceneStructs.h:171-175, vendored at path_tracer/external/include/stb_image.h).
Only tests/ may import it; the product decodes in C++ (cuda_pathtracer_amd/csrc/pt_jpeg.cpp).

Structure (different from the product's streaming decoder): the entropy-coded segments are
unstuffed and split at restart markers up front, Huffman codes are read through a 16-bit
look-ahead window over the whole bit string, blocks are collected first and then transformed all
at once with vectorised integer arithmetic.  The arithmetic itself is stb_image 2.06's:
  * coefficients: baseline (stb_image.h:1697-1747) and progressive per ITU T.81 G.1.2
    (stb :1749-1893: first DC/AC scans, refinement scans, EOB runs), dequantised with 8-bit tables;
  * integer IDCT (:1906-2004): 12-bit constants (x * 4096 + 0.5, float x), column pass keeping 2
    extra bits ((x + 512) >> 10), row pass (x + 65536 + (128 << 17)) >> 17, clamped to 0..255;
  * chroma upsampling (:2849-2911, :3030-3039) with load_jpeg_image's near/far row pairing
    (:3328-3362);
  * YCbCr -> RGB (:3070-3096): 20-bit fixed point with 12-bit coefficients, the green channel's
    Cb term truncated to a multiple of 2^16.
Parity: pinned by this restatement against the product byte for byte, and against PIL (a
different decoder, libjpeg) within a measured +-3 per texel; no stb_image build exists in this
image, so the stb output itself is not run here.
"""
from __future__ import annotations

import numpy as np

NATURAL = np.array([0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27,
                    20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58,
                    59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63] + [63] * 15)


class JpegError(ValueError):
    pass


def _table(counts, symbols):
    """16-bit prefix -> (symbol, code length) of a canonical Huffman code (T.81 Annex C)."""
    sym = np.full(1 << 16, -1, np.int32)
    ln = np.zeros(1 << 16, np.int32)
    code, k = 0, 0
    for length in range(1, 17):
        for _ in range(counts[length - 1]):
            lo = code << (16 - length)
            hi = (code + 1) << (16 - length)
            sym[lo:hi] = symbols[k]
            ln[lo:hi] = length
            code += 1
            k += 1
        code <<= 1
    return sym, ln


class _Bits:
    """A bit string with a 16-bit look-ahead window at every position (zeros past the end)."""

    def __init__(self, data: bytes):
        b = np.unpackbits(np.frombuffer(data, np.uint8)).astype(np.int64)
        b = np.concatenate([b, np.zeros(32, np.int64)])
        w = np.zeros(len(b) - 16, np.int64)
        for k in range(16):
            w += b[k:k + len(w)] << (15 - k)
        self.win = w.tolist()
        self.pos = 0

    def huff(self, tab):
        sym, ln = tab
        v = self.win[self.pos]
        if ln[v] == 0:
            raise JpegError("bad huffman code")
        self.pos += int(ln[v])
        return int(sym[v])

    def get(self, n):
        if n == 0:
            return 0
        v = self.win[self.pos] >> (16 - n)
        self.pos += n
        return v

    def extend(self, n):
        """receive(n) + extend (T.81 F.2.2.1): a leading 0 bit marks a negative value."""
        if n == 0:
            return 0
        v = self.get(n)
        return v if v >= (1 << (n - 1)) else v - ((1 << n) - 1)


def _segments(data: bytes):
    """Yield (marker, payload) for table/frame markers and ('SOS', header, [entropy intervals])."""
    if data[:2] != b"\xff\xd8":
        raise JpegError("no SOI")
    i = 2
    while i < len(data):
        while i < len(data) and data[i] != 0xFF:
            if data[i] != 0:
                raise JpegError("junk before marker")
            i += 1
        while i < len(data) and data[i] == 0xFF:
            i += 1
        if i >= len(data):
            break
        m = data[i]
        i += 1
        if m == 0xD9:
            return
        L = (data[i] << 8) | data[i + 1]
        payload = data[i + 2:i + L]
        i += L
        if m != 0xDA:
            yield m, payload
            continue
        intervals, cur = [], bytearray()   # entropy data up to the next non-RST marker
        while i < len(data):
            if data[i] == 0xFF and i + 1 < len(data) and data[i + 1] != 0:
                if 0xD0 <= data[i + 1] <= 0xD7:
                    intervals.append(bytes(cur))
                    cur = bytearray()
                    i += 2
                    continue
                break
            cur.append(data[i])
            i += 2 if data[i] == 0xFF else 1   # FF 00 -> FF
        intervals.append(bytes(cur))
        yield "SOS", (payload, intervals)
    raise JpegError("no EOI")


def _f2f(x):
    return int(np.float32(x) * np.float32(4096) + 0.5)


def _idct_1d(s):
    """stb's 1-D pass over axis 0 of s (8 x ...), int64; returns (x0..x3, t0..t3)."""
    p1 = (s[2] + s[6]) * _f2f(0.5411961)
    t2 = p1 + s[6] * _f2f(-1.847759065)
    t3 = p1 + s[2] * _f2f(0.765366865)
    e0, e1 = (s[0] + s[4]) * 4096, (s[0] - s[4]) * 4096
    x0, x3, x1, x2 = e0 + t3, e0 - t3, e1 + t2, e1 - t2
    o7, o5, o3, o1 = s[7], s[5], s[3], s[1]
    p3, p4, p1, p2 = o7 + o3, o5 + o1, o7 + o1, o5 + o3
    p5 = (p3 + p4) * _f2f(1.175875602)
    a0, a1, a2, a3 = o7 * _f2f(0.298631336), o5 * _f2f(2.053119869), o3 * _f2f(3.072711026), o1 * _f2f(1.501321110)
    p1 = p5 + p1 * _f2f(-0.899976223)
    p2 = p5 + p2 * _f2f(-2.562915447)
    p3 = p3 * _f2f(-1.961570560)
    p4 = p4 * _f2f(-0.390180644)
    return (x0, x1, x2, x3), (a0 + p1 + p3, a1 + p2 + p4, a2 + p2 + p3, a3 + p1 + p4)


def idct(blocks: np.ndarray) -> np.ndarray:
    """(n, 64) dequantised int16 coefficients (natural order) -> (n, 8, 8) uint8 samples."""
    d = blocks.astype(np.int64).reshape(-1, 8, 8).transpose(1, 2, 0)        # [row][col][n]
    (x0, x1, x2, x3), (t0, t1, t2, t3) = _idct_1d(d)                         # columns
    x0, x1, x2, x3 = x0 + 512, x1 + 512, x2 + 512, x3 + 512
    v = np.stack([(x0 + t3) >> 10, (x1 + t2) >> 10, (x2 + t1) >> 10, (x3 + t0) >> 10,
                  (x3 - t0) >> 10, (x2 - t1) >> 10, (x1 - t2) >> 10, (x0 - t3) >> 10])   # [row][col][n]
    (x0, x1, x2, x3), (t0, t1, t2, t3) = _idct_1d(v.transpose(1, 0, 2))       # rows
    b = 65536 + (128 << 17)
    x0, x1, x2, x3 = x0 + b, x1 + b, x2 + b, x3 + b
    o = np.stack([(x0 + t3) >> 17, (x1 + t2) >> 17, (x2 + t1) >> 17, (x3 + t0) >> 17,
                  (x3 - t0) >> 17, (x2 - t1) >> 17, (x1 - t2) >> 17, (x0 - t3) >> 17])   # [col][row][n]
    return np.clip(o, 0, 255).astype(np.uint8).transpose(2, 1, 0)


def _i16(x):
    return ((int(x) + 32768) & 0xFFFF) - 32768


def decode(data: bytes):
    """(height, width, components) uint8 array, as stbi_load(..., req_comp = 0) returns it."""
    q = {}
    dc_t, ac_t = {}, {}
    frame = None
    restart = 0
    coef = None
    for m, payload in _segments(data):
        if m == 0xDB:
            k = 0
            while k < len(payload):
                pq, tq = payload[k] >> 4, payload[k] & 15
                if pq != 0:
                    raise JpegError("16-bit DQT")
                t = np.zeros(64, np.int64)
                t[NATURAL[:64]] = np.frombuffer(payload[k + 1:k + 65], np.uint8)
                q[tq] = t
                k += 65
        elif m == 0xC4:
            k = 0
            while k < len(payload):
                tc, th = payload[k] >> 4, payload[k] & 15
                counts = list(payload[k + 1:k + 17])
                n = sum(counts)
                tab = _table(counts, list(payload[k + 17:k + 17 + n]))
                (dc_t if tc == 0 else ac_t)[th] = tab
                k += 17 + n
        elif m == 0xDD:
            restart = (payload[0] << 8) | payload[1]
        elif m in (0xC0, 0xC1, 0xC2):
            if payload[0] != 8:
                raise JpegError("8-bit only")
            H, W, nc = (payload[1] << 8) | payload[2], (payload[3] << 8) | payload[4], payload[5]
            comps = [dict(id=payload[6 + 3 * c], h=payload[7 + 3 * c] >> 4, v=payload[7 + 3 * c] & 15,
                          tq=payload[8 + 3 * c]) for c in range(nc)]
            hm, vm = max(c["h"] for c in comps), max(c["v"] for c in comps)
            mx, my = -(-W // (8 * hm)), -(-H // (8 * vm))
            for c in comps:
                c["x"], c["y"] = -(-W * c["h"] // hm), -(-H * c["v"] // vm)
                c["bw"], c["bh"] = mx * c["h"], my * c["v"]         # blocks per row / column (whole MCUs)
            frame = dict(H=H, W=W, comps=comps, hm=hm, vm=vm, mx=mx, my=my, progressive=m == 0xC2)
            coef = [np.zeros((c["bh"], c["bw"], 64), np.int64) for c in comps]
        elif m == "SOS":
            _scan(frame, coef, dc_t, ac_t, restart, *payload)
        elif 0xE0 <= m <= 0xEF or m == 0xFE:
            pass
        else:
            raise JpegError(f"unsupported marker {m:#x}")
    comps = frame["comps"]
    planes = []
    for c, cf in zip(comps, coef):
        deq = cf * q[c["tq"]]                    # stb: (short)(v * dequant) per coefficient
        deq = ((deq + 32768) & 0xFFFF) - 32768
        px = idct(deq.reshape(-1, 64)).reshape(c["bh"], c["bw"], 8, 8).transpose(0, 2, 1, 3)
        planes.append(px.reshape(c["bh"] * 8, c["bw"] * 8).astype(np.int64))
    H, W = frame["H"], frame["W"]
    rows = [_upsample(p, c, frame) for p, c in zip(planes, comps)]
    if len(comps) == 1:
        return rows[0][:, :W].astype(np.uint8)[..., None]
    y, cb, cr = (r[:, :W] for r in rows)
    fx = lambda x: int(np.float32(x) * np.float32(4096.0) + np.float32(0.5)) << 8   # noqa: E731
    yf = (y << 20) + (1 << 19)
    dr, db = cr - 128, cb - 128
    r = (yf + dr * fx(1.40200)) >> 20
    g = (yf + dr * -fx(0.71414) + ((db * -fx(0.34414)) & ~0xFFFF)) >> 20
    b = (yf + db * fx(1.77200)) >> 20
    return np.clip(np.stack([r, g, b], -1), 0, 255).astype(np.uint8)


def _upsample(p, c, frame):
    """The component plane at full resolution, img_y rows (stb_image.h:3328-3362)."""
    H, W = frame["H"], frame["W"]
    hs, vs = frame["hm"] // c["h"], frame["vm"] // c["v"]
    wl = -(-W // hs)
    last = c["y"] - 1
    j = np.arange(H)
    if vs == 2:   # output row j pairs low-res rows near = j//2 ... (ystep alternation)
        m = j // 2
        odd = (j % 2) == 1
        near = np.where(odd, m, np.minimum(m, last))
        far = np.where(odd, np.minimum(m + 1, last), np.maximum(m - 1, 0))
    else:
        near = far = np.minimum(j // vs, last)
    nr, fr = p[near, :wl], p[far, :wl]
    if hs == 1 and vs == 1:
        return nr
    if hs == 1 and vs == 2:
        return (3 * nr + fr + 2) >> 2
    if hs == 2 and vs == 1:
        out = np.zeros((H, 2 * wl), np.int64)
        if wl == 1:
            out[:, 0] = out[:, 1] = nr[:, 0]
            return out
        n3 = 3 * nr + 2
        out[:, 0] = nr[:, 0]
        out[:, 1] = (nr[:, 0] * 3 + nr[:, 1] + 2) >> 2
        out[:, 2:2 * wl - 2:2] = (n3[:, 1:wl - 1] + nr[:, 0:wl - 2]) >> 2
        out[:, 3:2 * wl - 2:2] = (n3[:, 1:wl - 1] + nr[:, 2:wl]) >> 2
        out[:, 2 * wl - 2] = (nr[:, wl - 2] * 3 + nr[:, wl - 1] + 2) >> 2
        out[:, 2 * wl - 1] = nr[:, wl - 1]
        return out
    if hs == 2 and vs == 2:
        t = 3 * nr + fr
        out = np.zeros((H, 2 * wl), np.int64)
        if wl == 1:
            out[:, 0] = out[:, 1] = (t[:, 0] + 2) >> 2
            return out
        out[:, 0] = (t[:, 0] + 2) >> 2
        out[:, 1:2 * wl - 1:2] = (3 * t[:, :-1] + t[:, 1:] + 8) >> 4
        out[:, 2:2 * wl - 1:2] = (3 * t[:, 1:] + t[:, :-1] + 8) >> 4
        out[:, 2 * wl - 1] = (t[:, -1] + 2) >> 2
        return out
    return np.repeat(nr, hs, axis=1)   # other ratios: nearest


def _scan(frame, coef, dc_t, ac_t, restart, header, intervals):
    comps = frame["comps"]
    ns = header[0]
    sc = []
    for k in range(ns):
        cid, tabs = header[1 + 2 * k], header[2 + 2 * k]
        ci = next(i for i, c in enumerate(comps) if c["id"] == cid)
        sc.append((ci, tabs >> 4, tabs & 15))
    ss, se, ah, al = header[1 + 2 * ns], header[2 + 2 * ns], header[3 + 2 * ns] >> 4, header[3 + 2 * ns] & 15
    prog = frame["progressive"]
    if not prog:
        ss, se, ah, al = 0, 63, 0, 0
    # the block visiting order: MCUs of interleaved scans, or the component's own grid
    if ns == 1:
        ci = sc[0][0]
        c = comps[ci]
        units = [[(ci, by, bx)] for by in range(-(-c["y"] // 8)) for bx in range(-(-c["x"] // 8))]
    else:
        units = [[(ci, my * comps[ci]["v"] + y, mx * comps[ci]["h"] + x) for ci, _, _ in sc
                  for y in range(comps[ci]["v"]) for x in range(comps[ci]["h"])]
                 for my in range(frame["my"]) for mx in range(frame["mx"])]
    per = restart if restart else len(units)
    tabs = {ci: (hd, ha) for ci, hd, ha in sc}
    for seg, start in enumerate(range(0, len(units), per)):
        if seg >= len(intervals):
            break
        bits = _Bits(intervals[seg])
        pred = {ci: 0 for ci, _, _ in sc}
        eob = 0
        for unit in units[start:start + per]:
            for ci, by, bx in unit:
                blk = coef[ci][by, bx]
                hd, ha = tabs[ci]
                if ss == 0:   # DC (baseline: the whole block)
                    if ah == 0:
                        t = bits.huff(dc_t[hd])
                        pred[ci] += bits.extend(t)
                        if prog:
                            blk[:] = 0
                            blk[0] = _i16(pred[ci] << al)
                        else:
                            blk[:] = 0
                            blk[0] = pred[ci]
                    elif bits.get(1):
                        blk[0] = _i16(blk[0] + (1 << al))
                    if prog:
                        continue
                    k = 1   # baseline AC
                    while k < 64:
                        rs = bits.huff(ac_t[ha])
                        r, s = rs >> 4, rs & 15
                        if s == 0:
                            if rs != 0xF0:
                                break
                            k += 16
                            continue
                        k += r
                        blk[NATURAL[k]] = bits.extend(s)
                        k += 1
                    continue
                eob = _prog_ac(bits, ac_t[ha], blk, ss, se, ah, al, eob)


def _prog_ac(bits, tab, blk, ss, se, ah, al, eob):
    if ah == 0:
        if eob:
            return eob - 1
        k = ss
        while k <= se:
            rs = bits.huff(tab)
            r, s = rs >> 4, rs & 15
            if s == 0:
                if r < 15:
                    return (1 << r) + bits.get(r) - 1
                k += 16
                continue
            k += r
            blk[NATURAL[k]] = _i16(bits.extend(s) << al)
            k += 1
        return 0
    p1 = 1 << al
    if eob:
        for k in range(ss, se + 1):
            z = NATURAL[k]
            if blk[z] != 0 and bits.get(1) and (blk[z] & p1) == 0:
                blk[z] += p1 if blk[z] > 0 else -p1
        return eob - 1
    k = ss
    new_eob = 0
    while k <= se:
        rs = bits.huff(tab)
        r, s = rs >> 4, rs & 15
        val = 0
        if s == 0:
            if r < 15:
                new_eob = (1 << r) - 1 + bits.get(r)
                r = 64
        else:
            val = p1 if bits.get(1) else -p1
        while k <= se:
            z = NATURAL[k]
            k += 1
            if blk[z] != 0:
                if bits.get(1) and (blk[z] & p1) == 0:
                    blk[z] += p1 if blk[z] > 0 else -p1
            else:
                if r == 0:
                    blk[z] = val
                    break
                r -= 1
        if new_eob:
            break
    return new_eob


def load(path) -> np.ndarray:
    with open(path, "rb") as f:
        return decode(f.read())
