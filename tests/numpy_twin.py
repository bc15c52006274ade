"""Vectorised numpy restatement of the reference hot path (test infrastructure).

An independent second restatement of acquisition.m / trackingCT.m in the
"MATLAB-like vectorised" style, used only to cross-check the C oracle on small
inputs (tests/test_oracle_numpy_twin.py) and to co-sign the golden vectors.
"""
import math

import numpy as np


def colon(a, d, b):
    """MATLAB a:d:b (MathWorks colonop construction)."""
    if d == 0 or (a < b and d < 0) or (b < a and d > 0):
        return np.zeros(0)
    tol = 2.0 * np.finfo(float).eps * max(abs(a), abs(b))
    sig = 1.0 if d > 0 else -1.0
    if a == math.floor(a) and d == 1:
        n = math.floor(b) - a
    elif a == math.floor(a) and d == math.floor(d):
        q = math.floor(a / d)
        r = a - q * d
        n = math.floor((b - r) / d) - q
    else:
        n = float(np.round((b - a) / d))
        if sig * (a + n * d - b) > tol:
            n -= 1
    n = int(n)
    c = a + n * d
    if sig * (c - b) > -tol:
        c = b
    v = np.zeros(n + 1)
    k = np.arange(0, n // 2 + 1, dtype=float)
    v[(1 + k - 1).astype(int)] = a + k * d
    v[(n + 1 - k - 1).astype(int)] = c - k * d
    if n % 2 == 0:
        v[n // 2] = (a + c) / 2
    return v


def ca_code(prn):
    g2s = [5, 6, 7, 8, 17, 18, 139, 140, 141, 251, 252, 254, 255, 256, 257, 258, 469, 470, 471,
           472, 473, 474, 509, 512, 513, 514, 515, 516, 859, 860, 861, 862]
    reg = -np.ones(10)
    g1 = np.zeros(1023)
    for i in range(1023):
        g1[i] = reg[9]
        sb = reg[2] * reg[9]
        reg[1:] = reg[:-1].copy()
        reg[0] = sb
    reg = -np.ones(10)
    g2 = np.zeros(1023)
    for i in range(1023):
        g2[i] = reg[9]
        sb = reg[1] * reg[2] * reg[5] * reg[7] * reg[8] * reg[9]
        reg[1:] = reg[:-1].copy()
        reg[0] = sb
    s = g2s[prn - 1]
    g2 = np.concatenate([g2[1023 - s:], g2[:1023 - s]])
    return -(g1 * g2)


def correlate_step(iq, n, remChip, codeFreq, Fs, carrierFreq, remPhase, ca, taps):
    """trackingCT.m:96-118 for one step (sums per tap, I then Q)."""
    raw = iq[0:2 * n:2].astype(float) + 1j * iq[1:2 * n:2].astype(float)
    Code = np.concatenate([[ca[-1]], ca, ca, ca, ca, ca, ca, ca, ca, ca, ca, [ca[0]]])
    d = codeFreq / Fs
    CarrTime = np.arange(0, n + 1) / Fs
    Wave = (2 * np.pi * (carrierFreq * CarrTime)) + remPhase
    carrsig = np.exp(1j * Wave[:n])
    prod = raw * carrsig
    I, Q = np.imag(prod), np.real(prod)
    out = []
    for s in taps:
        t = colon((0 + s) + remChip, d, ((n - 1) * d + s) + remChip)
        code = Code[np.ceil(t).astype(int)]
        out += [math.fsum(code * I), math.fsum(code * Q)]
    return np.array(out)


def read_samples(buf, dataPrecision, dataType, nsamp):
    """fread + the reference's sample forming (acquisition.m:28-37, trackingCT.m:84-93) on the
    record bytes `buf` (int8 view): int8 I/Q or real; int16 values de-interleaved into I/Q
    (whatever dataType says) minus each half's mean."""
    buf = np.asarray(buf, dtype=np.int8)
    if dataPrecision == 1:
        v = buf[: nsamp * dataType].astype(float)
        return v[0::2] + 1j * v[1::2] if dataType == 2 else v + 0j
    v = buf[: 2 * nsamp * dataType].view("<i2").astype(float)
    si, co = v[0::2], v[1::2]
    return (si - np.mean(si)) + 1j * (co - np.mean(co))


def acquisition(raw8, S, Fs, IF, fc, freqMin, freqStep, freqNum, datalen, prns):
    """acquisition.m:40-78 (peak search only) on int8 I/Q bytes or complex samples."""
    raw = raw8 if np.iscomplexobj(raw8) else raw8[0::2].astype(float) + 1j * raw8[1::2].astype(float)
    n = np.arange(1, S + 1)
    res = []
    for prn in prns:
        oc = np.concatenate([ca_code(prn), ca_code(prn)])
        scode = oc[np.ceil(n * (fc / Fs)).astype(int) - 1]
        C = np.fft.fft(scode)
        corr = np.zeros((freqNum, S))
        for idx in range(datalen):
            blk = raw[idx * S:(idx + 1) * S]
            for b in range(freqNum):
                carrier = np.exp(1j * 2 * np.pi * (IF + freqMin + freqStep * b) * n / Fs)
                corr[b] += np.abs(np.fft.ifft(C * np.conj(np.fft.fft(blk * carrier)))) ** 2
        fbin = int(np.argmax(corr.max(axis=1)))
        cp = int(np.argmax(corr.max(axis=0)))
        peak = corr.max()
        cs = math.ceil(Fs / fc)
        row = corr[fbin]
        idx = np.r_[np.arange(0, max(0, cp + 1 - cs)), np.arange(cp + cs, S)]
        snr = 10 * np.log10(peak ** 2 / np.mean(row[idx] ** 2))
        res.append((prn, fbin + 1, cp + 1, snr))
    return res
