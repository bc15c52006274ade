"""Synthetic IF scenarios — the recordings themselves are absent.

A scenario is a gnss_synth config: per SV a PRN, Doppler, code phase, carrier
phase, C/N0 and a 50 bps nav-bit stream; AWGN sigma 12 LSB; int8 I/Q at the
Opensky shape (Fs 58 MHz, IF 4.58 MHz) unless stated. The SVs of the Opensky
scenario sit at the golden acquisition result Acquired_Opensky_5000.mat
(codedelay, fineFreq - IF), so acquisition should report those values.

`generate_device` fills HBM with the HIP generator (bench: multi-GB records
without a PCIe upload); tests generate small records with the CPU twin in
oracle/ and pass the same bytes to both paths.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import abi

FL1 = 1575.42e6
FC = 1.023e6

# Acquired_Opensky_5000.mat (tests/golden/ref_acquired.json)
OPENSKY_SV = [3, 4, 16, 22, 26, 27, 31, 32]
OPENSKY_CODEDELAY = [3683, 12701, 26051, 2610, 57908, 49778, 39064, 20170]
OPENSKY_FINEFREQ = [4580990, 4576905, 4579695, 4581565, 4581835, 4576775, 4581045, 4583345]
OPENSKY_SNR = [18.09533691, 17.2935525, 26.4349007, 19.83213032, 27.20599355, 22.7205602,
               24.40169056, 22.19831875]
# nAcquired_Urban_5000.mat: IF = 0 (fineFreq is the Doppler); Fs unknown (26 MHz assumed)
URBAN_SV = [1, 3, 7, 11, 18, 22]
URBAN_CODEDELAY = [22742, 1154, 10811, 24851, 15362, 2050]
URBAN_DOPPLER = [1200, 4285, 365, 405, -365, 3315]


def scenario(svs, codedelays, dopplers, cn0s, *, Fs=58e6, IF=4.58e6, skip_ms=5000, sigma=12.0,
             seed=6102):
    """SVs placed so that the acquisition block starting at skip_ms sees
    codedelay (samples) and Doppler (Hz) for each PRN."""
    S = math.ceil(Fs * 1e-3)
    d0 = FC / Fs
    rng = np.random.Generator(np.random.PCG64(seed))
    cfg = abi.GnssSynth()
    cfg.Fs, cfg.IF, cfg.noise_sigma, cfg.seed = Fs, IF, sigma, seed
    cfg.n_sv = len(svs)
    n_ref = skip_ms * S - 1  # sample before the block start (block-relative n = 0)
    for i, (prn, cd, fd, cn0) in enumerate(zip(svs, codedelays, dopplers, cn0s)):
        crate = FC * (1.0 + fd / FL1) / Fs
        v = cfg.sv[i]
        v.prn = int(prn)
        v.doppler_hz = float(fd)
        v.code_phase0 = cd * d0 - n_ref * crate
        v.carr_phase0 = float(rng.random())
        v.cn0_dbhz = float(cn0)
        v.bit_seed = int(rng.integers(1, 2**62))
        v.bit_phase_chips = float(rng.random() * 20460.0)
    return cfg


def codedelays(cfg, skip_ms):
    """The code delays (samples, acquisition.m's codedelay convention) `scenario` placed each
    SV at, recovered from its code phase: the inverse of code_phase0 = cd*d0 - n_ref*crate."""
    S = math.ceil(cfg.Fs * 1e-3)
    d0 = FC / cfg.Fs
    n_ref = skip_ms * S - 1
    out = []
    for i in range(cfg.n_sv):
        v = cfg.sv[i]
        crate = FC * (1.0 + v.doppler_hz / FL1) / cfg.Fs
        out.append(int(round((v.code_phase0 + n_ref * crate) / d0)) % S)
    return out


def opensky(skip_ms=5000, seed=6102, cn0=None):
    cn0s = cn0 or [40.0 + (s - 17.0) * 0.8 for s in OPENSKY_SNR]
    dop = [f - 4.58e6 for f in OPENSKY_FINEFREQ]
    return scenario(OPENSKY_SV, OPENSKY_CODEDELAY, dop, cn0s, skip_ms=skip_ms, seed=seed)


def urban(skip_ms=5000, seed=6103, Fs=26e6):
    cn0s = [46.0, 44.0, 41.0, 42.0, 40.5, 40.0]
    return scenario(URBAN_SV, URBAN_CODEDELAY, URBAN_DOPPLER, cn0s, Fs=Fs, IF=0.0,
                    skip_ms=skip_ms, seed=seed)


def all_prn(n=32, skip_ms=0, seed=6105, Fs=58e6, IF=4.58e6):
    """Config 5: every PRN present, random code phases / Dopplers, 40-48 dB-Hz."""
    rng = np.random.Generator(np.random.PCG64(seed))
    S = math.ceil(Fs * 1e-3)
    svs = list(range(1, n + 1))
    cds = [int(x) for x in rng.integers(0, S, n)]
    dops = [float(x) for x in rng.uniform(-4000, 4000, n)]
    cn0s = [float(x) for x in rng.uniform(40, 48, n)]
    return scenario(svs, cds, dops, cn0s, Fs=Fs, IF=IF, skip_ms=skip_ms, seed=seed)


# The synthetic LNAV ephemeris of csrc/lnav.cpp (gnss_lnav_bits, gnss_synth_sv.lnav = 1):
# field -> (raw value, bits, signed, scale) as naviDecode_updated.m decodes it
LNAV_TOW0 = 390114  # TOW of the first subframe 1, s
LNAV_FIELDS = {
    "weeknum": (131 + 2048, 10, False, 1.0), "N": (0, 4, False, 1.0), "health": (0, 5, False, 1.0),
    "IODC": (56, 8, False, 1.0), "TGD": (4, 8, True, 2.0 ** -31), "toc": (24750, 16, False, 16.0),
    "af2": (0, 8, True, 2.0 ** -55), "af1": (65415, 16, True, 2.0 ** -43),
    "af0": (3497117, 22, True, 2.0 ** -31), "IODE2": (56, 8, False, 1.0),
    "Crs": (62011, 16, True, 2.0 ** -5), "deltan": (12325, 16, True, 2.0 ** -43, "pi"),
    "M0": (942312117, 32, True, 2.0 ** -31, "pi"), "Cuc": (65439, 16, True, 2.0 ** -29),
    "ecc": (33351524, 32, False, 2.0 ** -33), "Cus": (101, 16, True, 2.0 ** -29),
    "sqrta": (2702053453, 32, False, 2.0 ** -19), "toe": (24750, 16, False, 16.0),
    "Cic": (65522, 16, True, 2.0 ** -29), "omegae": (944858321, 32, True, 2.0 ** -31, "pi"),
    "Cis": (65502, 16, True, 2.0 ** -29), "i0": (663888912, 32, True, 2.0 ** -31, "pi"),
    "Crc": (8513, 16, True, 2.0 ** -5), "w": (683398911, 32, True, 2.0 ** -31, "pi"),
    "omegadot": (16776433, 24, True, 2.0 ** -43, "pi"), "IODE3": (56, 8, False, 1.0),
    "idot": (16336, 14, True, 2.0 ** -43, "pi"),
}


def lnav_expected(field: str) -> float:
    """The value naviDecode_updated.m decodes for a LNAV_FIELDS entry (bin2dec_GPSSDR /
    comp2dec semantics: two's complement on the field width, times 2^LSB, times pi)."""
    e = LNAV_FIELDS[field]
    raw, bits, signed, scale = e[:4]
    if field == "weeknum":
        return float(raw)
    v = raw - (1 << bits) if signed and raw >> (bits - 1) else raw
    out = float(v) * scale
    return out * math.pi if len(e) > 4 else out


def lnav_bits(nbits: int) -> np.ndarray:
    """gnss_lnav_bits: the transmitted bits (0/1) of the synthetic LNAV message."""
    out = np.zeros(nbits, dtype=np.int8)
    st = abi.load().gnss_lnav_bits(1, int(nbits), out.ctypes.data_as(C.c_void_p))
    if st != abi.OK:
        raise abi.GnssError(st, "gnss_lnav_bits")
    return out


def record_bytes(ms: float, Fs=58e6) -> int:
    return int(round(ms * math.ceil(Fs * 1e-3))) * 2


def generate_device(ctx, cfg, dev_record, sample0=0, nsamples=None):
    """Fill a DeviceRecord with samples [sample0, sample0+nsamples) (2 B each)."""
    n = dev_record.nbytes // 2 if nsamples is None else int(nsamples)
    ctx.check(ctx.lib.gnss_synth_if_device(ctx.h, C.byref(cfg), C.c_uint64(sample0),
                                           C.c_uint64(n), dev_record.ptr))
    return dev_record


def convert_record(iq8: np.ndarray, dataPrecision: int = 1, dataType: int = 2, *, scale: int = 64,
                   dc=(37, -23)) -> np.ndarray:
    """Byte image of the same scene in another record format (initParameters.m:36-37):
      (1, 2) int8 I/Q pairs (the input, unchanged);
      (1, 1) int8 real: the I byte of each pair (Re of the -(IF+fd) carrier still holds
             the SV at +-(IF+fd), the reference's carrier wipes the negative one);
      (2, 2) int16 I/Q: I*scale + dc[0], Q*scale + dc[1] (a DC offset the reference's
             per-read mean removal takes out, acquisition.m:28-32, trackingCT.m:84-88);
      (2, 1) int16 real values (the reference de-interleaves them as I/Q anyway).
    Returned as int8 bytes (little-endian int16 where dataPrecision is 2)."""
    iq8 = np.asarray(iq8, dtype=np.int8)
    i8, q8 = iq8[0::2], iq8[1::2]
    if dataPrecision == 1:
        return iq8.copy() if dataType == 2 else i8.copy()
    i16 = i8.astype(np.int16) * np.int16(scale) + np.int16(dc[0])
    if dataType == 1:
        return i16.astype("<i2").view(np.int8)
    q16 = q8.astype(np.int16) * np.int16(scale) + np.int16(dc[1])
    out = np.empty(2 * len(i16), dtype="<i2")
    out[0::2], out[1::2] = i16, q16
    return out.view(np.int8)
