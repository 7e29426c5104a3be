"""Minimal FLAC decoder for the bundled example audio (no third-party audio library offline).

The reference reads its examples with ``miniaudio.decode_file(path, nchannels=1, sample_rate=8000)``
(``tone/demo/read_audio.py:25-53``); miniaudio is not installed here.  The example files are mono
8 kHz 16-bit FLAC, so decoding is all that call does for them; this module decodes FLAC (STREAMINFO,
frame headers, CONSTANT / VERBATIM / FIXED / LPC subframes, partitioned Rice residuals, wasted
bits, stereo decorrelation) and checks the result against the MD5 the encoder stored in
STREAMINFO, which pins the decode bit-exactly.  Resampling / down-mixing are not implemented:
other rates or channel counts raise instead of silently differing from miniaudio.

Host-side input plumbing, not part of the acoustic hot path.
"""

from __future__ import annotations

import hashlib
from pathlib import Path

import numpy as np

__all__ = ["FlacError", "decode_flac", "read_audio"]


class FlacError(ValueError):
    pass


class _Bits:
    def __init__(self, data: bytes, byte_pos: int):
        self.d = data
        self.p = byte_pos * 8

    def read(self, n: int) -> int:
        if n == 0:
            return 0
        p = self.p
        b0 = p >> 3
        nb = ((p & 7) + n + 7) >> 3
        chunk = int.from_bytes(self.d[b0:b0 + nb], "big")
        self.p = p + n
        return (chunk >> (nb * 8 - (p & 7) - n)) & ((1 << n) - 1)

    def read_signed(self, n: int) -> int:
        v = self.read(n)
        return v - (1 << n) if n and v >> (n - 1) else v

    def unary(self) -> int:
        """Number of 0 bits before the next 1 bit (the 1 is consumed)."""
        d, p = self.d, self.p
        b = p >> 3
        cur = (d[b] << (p & 7)) & 0xFF
        if cur:
            z = 8 - cur.bit_length()
            self.p = p + z + 1
            return z
        count = 8 - (p & 7)
        b += 1
        while d[b] == 0:
            count += 8
            b += 1
        z = 8 - d[b].bit_length()
        self.p = (b << 3) + z + 1
        return count + z

    def align(self) -> None:
        self.p = (self.p + 7) & ~7


_FIXED = ([], [1], [2, -1], [3, -3, 1], [4, -6, 4, -1])
_RATES = (None, 88200, 176400, 192000, 8000, 16000, 22050, 24000, 32000, 44100, 48000, 96000)
_SIZES = (None, 8, 12, None, 16, 20, 24, 32)


def _residual(bits: _Bits, block: int, order: int) -> list:
    method = bits.read(2)
    if method > 1:
        raise FlacError(f"reserved residual coding method {method}")
    pbits, escape = (4, 15) if method == 0 else (5, 31)
    porder = bits.read(4)
    out = []
    for part in range(1 << porder):
        n = (block >> porder) - (order if part == 0 else 0)
        k = bits.read(pbits)
        if k == escape:
            w = bits.read(5)
            out.extend(bits.read_signed(w) for _ in range(n))
            continue
        for _ in range(n):
            u = (bits.unary() << k) | bits.read(k)
            out.append((u >> 1) ^ -(u & 1))
    return out


def _subframe(bits: _Bits, block: int, bps: int) -> list:
    if bits.read(1):
        raise FlacError("subframe padding bit set")
    kind = bits.read(6)
    wasted = 0
    if bits.read(1):
        wasted = bits.unary() + 1
        bps -= wasted
    if kind == 0:                                             # CONSTANT
        s = [bits.read_signed(bps)] * block
    elif kind == 1:                                           # VERBATIM
        s = [bits.read_signed(bps) for _ in range(block)]
    elif 8 <= kind <= 12:                                     # FIXED, order 0..4
        order = kind - 8
        s = [bits.read_signed(bps) for _ in range(order)]
        res = _residual(bits, block, order)
        c = _FIXED[order]
        for r in res:
            s.append(r + sum(cj * s[-1 - j] for j, cj in enumerate(c)))
    elif kind >= 32:                                          # LPC, order 1..32
        order = kind - 31
        s = [bits.read_signed(bps) for _ in range(order)]
        prec = bits.read(4) + 1
        if prec == 16:
            raise FlacError("invalid LPC coefficient precision")
        shift = bits.read_signed(5)
        if shift < 0:
            raise FlacError("negative LPC shift")
        c = [bits.read_signed(prec) for _ in range(order)]
        res = _residual(bits, block, order)
        for r in res:
            acc = 0
            for j, cj in enumerate(c):
                acc += cj * s[-1 - j]
            s.append(r + (acc >> shift))
    else:
        raise FlacError(f"reserved subframe type {kind}")
    return [v << wasted for v in s] if wasted else s


def decode_flac(data: bytes, verify_md5: bool = True) -> tuple[np.ndarray, int]:
    """FLAC bytes -> (samples int32 [n] or [n, channels], sample_rate)."""
    if data[:4] != b"fLaC":
        raise FlacError("not a FLAC stream")
    pos, info = 4, None
    while True:
        hdr = data[pos]
        n = int.from_bytes(data[pos + 1:pos + 4], "big")
        if hdr & 0x7F == 0:
            b = _Bits(data, pos + 4)
            b.read(16), b.read(16), b.read(24), b.read(24)
            info = {"rate": b.read(20), "channels": b.read(3) + 1, "bps": b.read(5) + 1, "total": b.read(36),
                    "md5": data[pos + 4 + 18:pos + 4 + 34]}
        pos += 4 + n
        if hdr & 0x80:
            break
    if info is None:
        raise FlacError("missing STREAMINFO")
    chans = [[] for _ in range(info["channels"])]
    bits = _Bits(data, pos)
    while len(chans[0]) < info["total"] and (bits.p >> 3) + 2 < len(data):
        if bits.read(14) != 0x3FFE:
            raise FlacError(f"lost frame sync at byte {bits.p // 8}")
        bits.read(2)
        bs_code, sr_code, ch_code, ss_code = bits.read(4), bits.read(4), bits.read(4), bits.read(3)
        bits.read(1)
        first = bits.read(8)                                  # UTF-8 coded frame / sample number
        extra = 0
        while first & (0x80 >> extra):
            extra += 1
        for _ in range(max(extra - 1, 0)):
            bits.read(8)
        if bs_code == 1:
            block = 192
        elif 2 <= bs_code <= 5:
            block = 576 << (bs_code - 2)
        elif bs_code == 6:
            block = bits.read(8) + 1
        elif bs_code == 7:
            block = bits.read(16) + 1
        elif bs_code >= 8:
            block = 256 << (bs_code - 8)
        else:
            raise FlacError("reserved block size")
        if sr_code == 12:
            bits.read(8)
        elif sr_code in (13, 14):
            bits.read(16)
        bps = info["bps"] if ss_code == 0 else _SIZES[ss_code]
        if bps is None:
            raise FlacError("reserved sample size")
        bits.read(8)                                          # header CRC-8 (the stream MD5 is checked)
        nch = ch_code + 1 if ch_code < 8 else 2
        sub = []
        for c in range(nch):
            side = (ch_code == 8 and c == 1) or (ch_code == 9 and c == 0) or (ch_code == 10 and c == 1)
            sub.append(_subframe(bits, block, bps + (1 if side else 0)))
        if ch_code == 8:                                      # left / side
            sub[1] = [l - s for l, s in zip(sub[0], sub[1])]
        elif ch_code == 9:                                    # side / right
            sub[0] = [s + r for s, r in zip(sub[0], sub[1])]
        elif ch_code == 10:                                   # mid / side
            m_s = [((m << 1) | (s & 1), s) for m, s in zip(sub[0], sub[1])]
            sub[0] = [(m + s) >> 1 for m, s in m_s]
            sub[1] = [(m - s) >> 1 for m, s in m_s]
        for c in range(nch):
            chans[c].extend(sub[c])
        bits.align()
        bits.read(16)                                         # frame CRC-16
    pcm = np.array(chans, dtype=np.int64).T[: info["total"]]
    if verify_md5 and any(info["md5"]):
        width = (info["bps"] + 7) // 8
        raw = b"".join(int(v).to_bytes(width, "little", signed=True) for v in pcm.reshape(-1)) if width != 2 else \
            pcm.astype("<i2").tobytes()
        if hashlib.md5(raw).digest() != info["md5"]:
            raise FlacError("decoded samples do not match the STREAMINFO MD5")
    out = pcm.astype(np.int32)
    return (out[:, 0] if info["channels"] == 1 else out), info["rate"]


def read_audio(path) -> np.ndarray:
    """Mono 8 kHz FLAC -> int32 samples, as ``tone/demo/read_audio.py:25-53`` returns them."""
    pcm, rate = decode_flac(Path(path).read_bytes())
    if rate != 8000 or pcm.ndim != 1:
        raise FlacError(f"{path}: {rate} Hz, {1 if pcm.ndim == 1 else pcm.shape[1]} channels; only mono 8 kHz "
                        "is decoded here (the reference resamples with miniaudio)")
    return pcm
