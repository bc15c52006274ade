"""Host-side mirror of the reference's MATLAB interface for the hot path.

    [file, signal, acq, track, solu, cmn] = initParameters()      initParameters.m:1-85
    Acquired = acquisition(file, signal, acq)                      acquisition.m:1
    [TckResultCT, CN0_Eph, countinx] = trackingCT(file, signal, track, Acquired)
                                                                   trackingCT.m:1
    [TckResultCT_pos, CN0_CT] = trackingCT_POS(file, signal, track, Acquired, countinx)
                                   tracking loop of trackingCT_POS_updated.m:1-413
    [ephemeris, ALLTckResult, for_prest] = naviDecode_updated(Acquired, ALLTckResult)
                                                                   naviDecode_updated.m:1

Same names, same struct fields, same argument meaning; the work happens in the
HIP C-ABI library (abi.py). Differences forced by the language are documented
per function. Errors follow the reference: nothing acquired -> empty Acquired
(acquisition.m:84-85); "Not enough raw data" -> TckResultCT = [] (returned as
an empty StructArray); conditions where MATLAB raises -> GnssError.
"""
from __future__ import annotations

import ctypes as C
import math
from types import SimpleNamespace

import numpy as np

from . import abi


# ---------------------------------------------------------------------------
# initParameters.m
# ---------------------------------------------------------------------------
def initParameters(fileRoute: str | None = None):
    """Struct surface of initParameters.m:1-85 (Opensky defaults).

    file.fid (a MATLAB file handle opened at :35) has no Python equivalent: the
    core does positioned reads of file.fileRoute, or uses file.data (an int8
    numpy record held in host memory) / file.dev (a DeviceRecord in HBM).
    """
    file = SimpleNamespace(fileName="Opensky", fileRoute=fileRoute, skip=5000, skiptimeVT=100,
                           dataType=2, dataPrecision=1, data=None, dev=None)
    signal = SimpleNamespace(IF=4.58e6, Fs=58e6, Fc=1575.42e6, codeFreqBasis=1.023e6, ms=1e-3)
    signal.Sample = math.ceil(signal.Fs * signal.ms)
    signal.codelength = signal.codeFreqBasis * signal.ms
    acq = SimpleNamespace(prnList=list(range(1, 33)), freqStep=500, freqMin=-10000, datalen=20, L=10)
    acq.freqNum = int(2 * abs(acq.freqMin) / acq.freqStep + 1)
    track = SimpleNamespace(CorrelatorSpacing=0.5, DLLBW=2, DLLDamp=0.707, DLLGain=0.1, PLLBW=15,
                            PLLDamp=0.707, PLLGain=0.25, msToProcessCT_1ms=1000,
                            msToProcessCT_10ms=40000, ctPOS=3000, msToProcessVT=5000, pdi=1)
    solu = SimpleNamespace(iniPos=[22.328444770087565 / 180 * math.pi,
                                   114.1713630049711 / 180 * math.pi, 4],
                           navSolPeriod=20, mode=2)
    cmn = SimpleNamespace(doy=171, vtEnable=1, mltCorrON=[1, 0], cSpeed=299792458, equip="stereo")
    return file, signal, acq, track, solu, cmn


# ---------------------------------------------------------------------------
# device context
# ---------------------------------------------------------------------------
class Context:
    """One gnss_ctx on one HIP device (stream, rocFFT plans, device buffers), or with
    `devices` a multi-device context (gnss_ctx_create_multi): acquisition and trackingCT deal
    their PRNs / channels round-robin over one member context per entry (a device may repeat)
    and merge the rows, bit-identical to one context; device-resident records and outputs
    belong to devices[0]."""

    def __init__(self, device: int = 0, devices=None):
        self.lib = abi.load()
        h = C.c_void_p()
        if devices is not None:
            devs = [int(d) for d in devices]
            arr = (C.c_int * len(devs))(*devs)
            st = self.lib.gnss_ctx_create_multi(arr, len(devs), C.byref(h))
            if st != abi.OK:
                raise abi.GnssError(st, f"gnss_ctx_create_multi(devices={devs}) failed")
            device = devs[0]
        else:
            st = self.lib.gnss_ctx_create(int(device), C.byref(h))
            if st != abi.OK:
                raise abi.GnssError(st, f"gnss_ctx_create(device={device}) failed")
        self.h = h
        self.device = device
        self.devices = list(devices) if devices is not None else [device]

    @property
    def members(self) -> int:
        return int(self.lib.gnss_ctx_members(self.h))

    def close(self):
        if getattr(self, "h", None):
            self.lib.gnss_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, st):
        if st != abi.OK:
            raise abi.GnssError(st, (self.lib.gnss_last_error(self.h) or b"").decode())
        return st

    def timing(self) -> dict:
        t = abi.GnssTiming()
        self.check(self.lib.gnss_last_timing(self.h, C.byref(t)))
        return {f: getattr(t, f) for f, _ in abi.GnssTiming._fields_}

    def set_profiling(self, on: bool):
        self.check(self.lib.gnss_ctx_set_profiling(self.h, 1 if on else 0))

    def set_window(self, nbytes: int):
        """Streaming: at most nbytes of IF resident in HBM per trackingCT call (0: the whole
        read range), gnss_ctx_set_window."""
        self.check(self.lib.gnss_ctx_set_window(self.h, int(nbytes)))

    def set_option(self, key: int, value: int):
        """Test hook: force one engine path (abi.OPT_*, gnss_ctx_set_option)."""
        self.check(self.lib.gnss_ctx_set_option(self.h, int(key), int(value)))

    def drop_record(self, dev=None):
        """Multi-device contexts: drop the members' resident copies of a device record (a
        DeviceRecord, a device pointer, or None for all), gnss_ctx_drop_record; needed only when
        the record's bytes were rewritten outside the library."""
        if dev is None:
            ptr = None
        else:
            v = getattr(dev, "ptr", dev)
            ptr = v.value if isinstance(v, C.c_void_p) else int(v)
        self.check(self.lib.gnss_ctx_drop_record(self.h, C.c_void_p(ptr)))

    @property
    def resident_records(self) -> int:
        """Resident record copies held by the members (gnss_ctx_resident_records)."""
        return int(self.lib.gnss_ctx_resident_records(self.h))

    def set_acq_precision(self, fp64: bool):
        """Acquisition correlation at fp64 (the reference's precision, default) or the fp32
        fast mode (gnss_ctx_set_acq_precision)."""
        self.check(self.lib.gnss_ctx_set_acq_precision(self.h, 1 if fp64 else 0))


class DeviceRecord:
    """An IF record resident in this context's HBM (bytes = file bytes)."""

    def __init__(self, ctx: Context, nbytes: int):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        ctx.check(ctx.lib.gnss_dev_alloc(ctx.h, C.c_uint64(self.nbytes), C.byref(p)))
        self.ptr = p

    @classmethod
    def from_host(cls, ctx: Context, data: np.ndarray):
        data = np.ascontiguousarray(data, dtype=np.int8)
        r = cls(ctx, data.nbytes)
        ctx.check(ctx.lib.gnss_dev_upload(ctx.h, r.ptr, data.ctypes.data_as(C.c_void_p),
                                          C.c_uint64(data.nbytes)))
        return r

    def upload(self, data: np.ndarray, offset: int = 0):
        """Host bytes into the record at `offset` (gnss_dev_upload; a multi-device context's
        members drop their resident copies of the record)."""
        data = np.ascontiguousarray(data, dtype=np.int8)
        dst = C.c_void_p(self.ptr.value + int(offset))
        self.ctx.check(self.ctx.lib.gnss_dev_upload(self.ctx.h, dst, data.ctypes.data_as(C.c_void_p),
                                                    C.c_uint64(data.nbytes)))

    def download(self, offset: int = 0, nbytes: int | None = None) -> np.ndarray:
        n = self.nbytes - offset if nbytes is None else int(nbytes)
        out = np.empty(n, dtype=np.int8)
        src = C.c_void_p(self.ptr.value + int(offset))
        self.ctx.check(self.ctx.lib.gnss_dev_download(self.ctx.h, out.ctypes.data_as(C.c_void_p),
                                                      src, C.c_uint64(n)))
        return out

    def free(self):
        if self.ptr:
            self.ctx.lib.gnss_dev_free(self.ctx.h, self.ptr)
            self.ptr = None


_default_ctx: Context | None = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


# ---------------------------------------------------------------------------
# struct marshalling
# ---------------------------------------------------------------------------
def to_c_file(file):
    f = abi.GnssFile()
    keep = []
    path = getattr(file, "fileRoute", None)
    data = getattr(file, "data", None)
    dev = getattr(file, "dev", None)
    if dev is not None:
        f.dev_data = dev.ptr
        f.nbytes = dev.nbytes
    elif data is not None:
        # the record's byte image (an int16 array is passed through as its bytes)
        arr = np.ascontiguousarray(data) if isinstance(data, np.ndarray) else np.asarray(data, np.int8)
        arr = arr.reshape(-1).view(np.int8)
        keep.append(arr)
        f.data = arr.ctypes.data
        f.nbytes = arr.nbytes
    elif path:
        f.path = str(path).encode()
    else:
        raise abi.GnssError(abi.EARG, "file has no fileRoute, data or dev record")
    f.skip = int(file.skip)
    f.dataType = int(file.dataType)
    f.dataPrecision = int(file.dataPrecision)
    return f, keep


def to_c_signal(signal):
    s = abi.GnssSignal()
    s.IF, s.Fs, s.codeFreqBasis, s.ms = signal.IF, signal.Fs, signal.codeFreqBasis, signal.ms
    s.Sample = int(signal.Sample)
    s.codelength = signal.codelength
    return s


def to_c_acq(acq, prn_list=None):
    a = abi.GnssAcq()
    a.freqNum, a.freqMin, a.freqStep = int(acq.freqNum), float(acq.freqMin), float(acq.freqStep)
    a.datalen, a.L = int(acq.datalen), int(acq.L)
    keep = []
    if prn_list is not None:
        arr = np.ascontiguousarray(prn_list, dtype=np.int32)
        keep.append(arr)
        a.n_prn = len(arr)
        a.prn_list = arr.ctypes.data_as(C.POINTER(C.c_int32))
    return a, keep


def to_c_acquired(Acquired):
    a = abi.GnssAcquired()
    n = len(Acquired.sv)
    a.n = n
    for i in range(n):
        a.sv[i] = int(Acquired.sv[i])
        a.SNR[i] = float(Acquired.SNR[i])
        a.Doppler[i] = float(Acquired.Doppler[i])
        a.codedelay[i] = int(Acquired.codedelay[i])
        a.fineFreq[i] = float(Acquired.fineFreq[i])
    return a


def from_c_acquired(a) -> SimpleNamespace:
    n = a.n
    return SimpleNamespace(sv=np.array(a.sv[:n], dtype=np.int64),
                           SNR=np.array(a.SNR[:n]), Doppler=np.array(a.Doppler[:n]),
                           codedelay=np.array(a.codedelay[:n], dtype=np.int64),
                           fineFreq=np.array(a.fineFreq[:n]))


def to_c_track(track, taps=None, channels=None):
    t = abi.GnssTrack()
    for f in ["CorrelatorSpacing", "DLLBW", "DLLDamp", "DLLGain", "PLLBW", "PLLDamp", "PLLGain"]:
        setattr(t, f, float(getattr(track, f)))
    t.msToProcessCT_1ms = int(track.msToProcessCT_1ms)
    t.msToProcessCT_10ms = int(track.msToProcessCT_10ms)
    keep = []
    if taps is not None:
        arr = np.ascontiguousarray(taps, dtype=np.float64)
        keep.append(arr)
        t.n_taps = len(arr)
        t.tap_offsets = arr.ctypes.data_as(C.POINTER(C.c_double))
    if channels is not None:
        arr = np.ascontiguousarray(channels, dtype=np.int32)
        keep.append(arr)
        t.n_chan = len(arr)
        t.chan = arr.ctypes.data_as(C.POINTER(C.c_int32))
    return t, keep


class TrackOutBuffers:
    """Caller-allocated trackingCT outputs (see gnss_track_out in the header)."""

    def __init__(self, nsv: int, track, ntaps: int = 0, ctPOS: int | None = None):
        self.max_len = int(track.msToProcessCT_1ms) + 19 + int(track.msToProcessCT_10ms)
        if ctPOS is not None:  # trackingCT_POS_updated: one row per step
            self.max_len = int(ctPOS)
        self.rec = np.zeros((nsv, abi.NFIELDS, self.max_len))
        self.taps = np.zeros((nsv, 2, ntaps, self.max_len)) if ntaps else None
        self.len = np.zeros(nsv, dtype=np.int64)
        self.countinx = np.zeros(nsv, dtype=np.int32)
        self.cn0_cap = max(int(track.msToProcessCT_1ms) + 19, int(track.msToProcessCT_10ms) // 10) // 20 + 1
        if ctPOS is not None:
            self.cn0_cap = int(ctPOS) // 20 + 1
        self.CN0 = np.zeros((self.cn0_cap, nsv))
        o = abi.GnssTrackOut()
        o.max_len = self.max_len
        o.rec = self.rec.ctypes.data_as(C.POINTER(C.c_double))
        o.taps = self.taps.ctypes.data_as(C.POINTER(C.c_double)) if ntaps else None
        o.len = self.len.ctypes.data_as(C.POINTER(C.c_int64))
        o.countinx = self.countinx.ctypes.data_as(C.POINTER(C.c_int32))
        o.CN0_Eph = self.CN0.ctypes.data_as(C.POINTER(C.c_double))
        o.cn0_cap = self.cn0_cap
        self.c = o
        self.shape = (nsv, self.max_len, ntaps, self.cn0_cap)

    def fits(self, nsv: int, track, ntaps: int) -> bool:
        max_len = int(track.msToProcessCT_1ms) + 19 + int(track.msToProcessCT_10ms)
        cn0_cap = max(int(track.msToProcessCT_1ms) + 19, int(track.msToProcessCT_10ms) // 10) // 20 + 1
        return self.shape == (nsv, max_len, ntaps, cn0_cap)


class DeviceTrackOutBuffers(TrackOutBuffers):
    """TrackOutBuffers whose rec / taps live in HBM (gnss_track_out.flags = GNSS_OUT_DEVICE):
    torch float64 tensors on `device`, filled by the library's expansion kernel; len,
    countinx and CN0 stay host arrays. The multi-GPU path all-gathers these rows over
    RCCL without a host round trip (dist.gather_tracking_rows_device)."""

    def __init__(self, nsv: int, track, ntaps: int = 0, device="cuda:0", ctPOS: int | None = None):
        torch = abi.require_torch()
        super().__init__(nsv, track, 0, ctPOS)
        self.device = torch.device(device)
        self.rec = torch.zeros((nsv, abi.NFIELDS, self.max_len), dtype=torch.float64, device=self.device)
        self.taps = (torch.zeros((nsv, 2, ntaps, self.max_len), dtype=torch.float64, device=self.device)
                     if ntaps else None)
        self.c.rec = C.cast(C.c_void_p(self.rec.data_ptr()), C.POINTER(C.c_double))
        self.c.taps = C.cast(C.c_void_p(self.taps.data_ptr()), C.POINTER(C.c_double)) if ntaps else None
        self.c.flags = abi.OUT_DEVICE
        self.shape = (nsv, self.max_len, ntaps, self.cn0_cap)

    def sync_producer(self):
        """The library writes on its own stream: torch's pending work on these tensors
        (allocation fill, an all-gather) must be done first."""
        import torch
        torch.cuda.current_stream(self.device).synchronize()

    def host(self) -> TrackOutBuffers:
        """A host copy (TrackOutBuffers) of the same result."""
        h = TrackOutBuffers.__new__(TrackOutBuffers)
        h.__dict__.update({k: v for k, v in self.__dict__.items() if k not in ("device",)})
        h.rec = self.rec.cpu().numpy()
        h.taps = self.taps.cpu().numpy() if self.taps is not None else None
        return h


class StructArray:
    """MATLAB struct array indexed by PRN: TckResultCT(prn).P_i (trackingCT.m:153)."""

    def __init__(self, entries: dict):
        self._e = entries

    def __call__(self, prn):
        return self._e[int(prn)]

    def __len__(self):
        return max(self._e) if self._e else 0

    def __bool__(self):
        return bool(self._e)

    def prns(self):
        return sorted(self._e)


def build_tck_result(Acquired, buf: TrackOutBuffers, channels=None, fields=None) -> StructArray:
    entries = {}
    chans = range(len(Acquired.sv)) if channels is None else channels
    fields = fields or abi.FIELDS
    for c in chans:
        n = int(buf.len[c])
        e = SimpleNamespace(**{f: buf.rec[c, k, :n].copy() for k, f in enumerate(fields)})
        if buf.taps is not None:
            e.taps_i = buf.taps[c, 0, :, :n].copy()
            e.taps_q = buf.taps[c, 1, :, :n].copy()
        entries[int(Acquired.sv[c])] = e
    return StructArray(entries)


# ---------------------------------------------------------------------------
# acquisition.m / trackingCT.m
# ---------------------------------------------------------------------------
def acquisition(file, signal, acq, *, ctx: Context | None = None, prn_list=None,
                diag: bool = False):
    """acquisition.m:1-127 on the GPU.

    Like the reference, acq.prnList is ignored (acquisition.m:47 hard-codes 1:32,
    quirk A.1); `prn_list` selects PRNs explicitly (config 1: [3]; rank sharding).
    Returns Acquired (fields sv, SNR, Doppler, codedelay, fineFreq as row vectors),
    plus the per-PRN detector diagnostics when diag=True.
    """
    ctx = ctx or default_context()
    f, k1 = to_c_file(file)
    s = to_c_signal(signal)
    a, k2 = to_c_acq(acq, prn_list)
    out = abi.GnssAcquired()
    dg = abi.GnssAcqDiag()
    st = ctx.lib.gnss_acquisition(ctx.h, C.byref(f), C.byref(s), C.byref(a), C.byref(out),
                                  C.byref(dg))
    if st not in (abi.OK, abi.ENODATA):
        ctx.check(st)
    if st == abi.ENODATA:
        print("No satellites acquired. Check parameter settings ... \n")
    res = from_c_acquired(out)
    if diag:
        n = dg.n
        d = SimpleNamespace(prn=np.array(dg.prn[:n]), SNR=np.array(dg.SNR[:n]),
                            fbin=np.array(dg.fbin[:n]), codePhase=np.array(dg.codePhase[:n]),
                            peak=np.array(dg.peak[:n]), peak2=np.array(dg.peak2[:n]))
        return res, d
    return res


def trackingCT(file, signal, track, Acquired, *, ctx: Context | None = None, taps=None,
               channels=None, save_countinx: str | None = None, raw: bool = False,
               out: "TrackOutBuffers | None" = None):
    """trackingCT.m:1-530 on the GPU -> (TckResultCT, CN0_Eph, countinx).

    TckResultCT is indexed by PRN (TckResultCT(prn).P_i), CN0_Eph is
    cn0_rows x nsv, countinx is 1 x nsv. `taps` enables the multi-correlator ACF
    taps (config 5); `channels` tracks a subset (multi-GPU shard). The side file
    countinx.mat of trackingCT.m:530 is written only when save_countinx names it.
    With raw=True the TrackOutBuffers are returned instead of the structs; `out` reuses
    a TrackOutBuffers of the same shape from an earlier call (no 10s of MB allocated and
    freed per call; rows of channels outside `channels` keep their old contents).
    """
    ctx = ctx or default_context()
    nsv = len(Acquired.sv)
    f, k1 = to_c_file(file)
    s = to_c_signal(signal)
    t, k2 = to_c_track(track, taps, channels)
    a = to_c_acquired(Acquired)
    ntaps = 0 if taps is None else len(taps)
    if out is not None and out.fits(nsv, track, ntaps):
        buf = out
        buf.len[:] = 0
        buf.countinx[:] = 0
    else:
        buf = TrackOutBuffers(nsv, track, ntaps)
    if isinstance(buf, DeviceTrackOutBuffers):
        buf.sync_producer()
    st = ctx.lib.gnss_tracking_ct(ctx.h, C.byref(f), C.byref(s), C.byref(t), C.byref(a),
                                  C.byref(buf.c))
    if st == abi.ENODATA:
        print("Not enough raw data  \n")
        return StructArray({}), np.zeros((0, nsv)), buf.countinx.astype(np.int64)
    ctx.check(st)
    if raw:
        return buf
    countinx = buf.countinx.astype(np.int64)
    if save_countinx:
        import scipy.io as sio
        sio.savemat(save_countinx, {"countinx": countinx.reshape(1, -1)})
    cn0 = buf.CN0[: buf.c.cn0_rows].copy()
    hb = buf.host() if isinstance(buf, DeviceTrackOutBuffers) else buf
    return build_tck_result(Acquired, hb, channels), cn0, countinx


def trackingCT_POS(file, signal, track, Acquired, countinx, *, ctx: Context | None = None,
                   channels=None, raw: bool = False):
    """The tracking loop of trackingCT_POS_updated.m (:92-144, :179-413) on the GPU ->
    (TckResultCT_pos, CN0_CT).

    The reference reads `countinx` from countinx.mat (:29) and indexes it by the channel's
    position in Acquired (quirk A.17); pass that vector here. track.ctPOS is the step count
    (datalength, :50). The positioning half of the reference function (pseudoranges,
    least squares, :420-565) is out of scope: TckResultCT_pos carries the fields of
    :273-292 (E_i ... delayValue, absoluteSampleCodedelay) per PRN, one row per step.
    """
    ctx = ctx or default_context()
    nsv = len(Acquired.sv)
    f, k1 = to_c_file(file)
    s = to_c_signal(signal)
    t, k2 = to_c_track(track, None, channels)
    a = to_c_acquired(Acquired)
    cx = np.ascontiguousarray(np.asarray(countinx).reshape(-1)[:nsv], dtype=np.int32)
    ctPOS = int(track.ctPOS)
    buf = TrackOutBuffers(nsv, track, 0, ctPOS=ctPOS)
    st = ctx.lib.gnss_tracking_ct_pos(ctx.h, C.byref(f), C.byref(s), C.byref(t), C.byref(a),
                                      ctPOS, cx.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(buf.c))
    ctx.check(st)
    if raw:
        return buf
    cn0 = buf.CN0[: buf.c.cn0_rows].copy()
    return build_tck_result(Acquired, buf, channels, abi.FIELDS_POS), cn0


def mc_result(Acquired, buf: TrackOutBuffers, channels=None, fields=None) -> StructArray:
    """TckResultCT_mltCorr: the loop fields plus every tap under the reference's names
    (E_i_060 ... P_i ... L_q060, trackingCT_POS_updated_multicorrelator.m:374-439,
    trackingCT_multiCorr-GIVEN.m:248-286)."""
    res = build_tck_result(Acquired, buf, channels, fields or abi.FIELDS_POS)
    for prn in res.prns():
        e = res(prn)
        for k, name in enumerate(abi.MC_TAP_NAMES):
            setattr(e, name.format("i"), e.taps_i[k])
            setattr(e, name.format("q"), e.taps_q[k])
    return res


def trackingCT_POS_updated_multicorrelator(file, signal, track, Acquired, *,
                                           ctx: Context | None = None, channels=None,
                                           raw: bool = False):
    """The tracking loop of trackingCT_POS_updated_multicorrelator.m (:41-136, :170-440) on
    the GPU -> (TckResultCT_mltCorr, CN0_CT).

    track.msPosCT (datalength, :49; initParameters.m does not define it, the caller sets
    it) and track.pdi (:46, 1 or 10) give msPosCT/pdi steps, every one at that pdi. The 25
    taps at Spacing = 0.6:-0.05:-0.6 are all recorded; E/P/L = Spacing(3)/(13)/(23) drive
    the loops. The positioning half (:446-590) is out of scope.
    """
    ctx = ctx or default_context()
    nsv = len(Acquired.sv)
    f, k1 = to_c_file(file)
    s = to_c_signal(signal)
    t, k2 = to_c_track(track, None, channels)
    a = to_c_acquired(Acquired)
    msPosCT, pdi = int(track.msPosCT), int(track.pdi)
    nsteps = msPosCT // pdi if pdi > 0 else 0
    buf = TrackOutBuffers(nsv, track, abi.MC_TAPS, ctPOS=max(nsteps, 1))
    st = ctx.lib.gnss_tracking_ct_mc(ctx.h, C.byref(f), C.byref(s), C.byref(t), C.byref(a),
                                     msPosCT, pdi, C.byref(buf.c))
    ctx.check(st)
    if raw:
        return buf
    cn0 = buf.CN0[: buf.c.cn0_rows].copy()
    return mc_result(Acquired, buf, channels), cn0


def trackingCT_multiCorr(file, signal, track, Acquired, *, datalength: int = 50000,
                         ctx: Context | None = None, raw: bool = False):
    """trackingCT_multiCorr-GIVEN.m (function trackingCT_multiCorr) on the GPU ->
    (TckResultCT, CN0_CT).

    `datalength` 1-ms steps per channel (:27 hard-codes 50000) from fseek(Sample - codedelay
    - 1 + skip*Sample) (:57), trackingCT.m's loop with ceil numSample on the 25 taps
    Spacing = -0.6:0.05:0.6. TckResultCT(prn) carries the trackingCT field names of :287-297
    plus E_i_060 ... L_q060; codedelay keeps the reference's linear sum over one shared
    nsv x datalength delayValue matrix (earlier channels' rows included).
    """
    ctx = ctx or default_context()
    nsv = len(Acquired.sv)
    f, k1 = to_c_file(file)
    s = to_c_signal(signal)
    t, k2 = to_c_track(track, None, None)
    a = to_c_acquired(Acquired)
    buf = TrackOutBuffers(nsv, track, abi.MC_TAPS, ctPOS=max(int(datalength), 1))
    st = ctx.lib.gnss_tracking_ct_multicorr(ctx.h, C.byref(f), C.byref(s), C.byref(t), C.byref(a),
                                            int(datalength), C.byref(buf.c))
    ctx.check(st)
    if raw:
        return buf
    return mc_result(Acquired, buf, None, abi.FIELDS), buf.CN0[: buf.c.cn0_rows].copy()


def naviDecode_updated(Acquired, ALLTckResult, *, eph_cap: int = 512):
    """naviDecode_updated.m:1-253 -> (ephemeris, ALLTckResult, for_prest).

    ALLTckResult(prn).P_i is read for every PRN of Acquired.sv, in that order (the
    reference's channel order matters: its bit arrays carry over between channels).
    ephemeris(prn) has the ini_eph.m fields as row vectors plus updateflag; for_prest.nav1
    / for_prest.sfb1 are indexed by PRN like the MATLAB vectors (nav1 has max(sv) entries,
    sfb1 ends at the last PRN that decoded a subframe 1). ALLTckResult is returned as given
    with .sfb1 added per PRN (the reference's second output). Host code (csrc/navdecode.cpp).
    """
    lib = abi.load()
    sv = [int(x) for x in Acquired.sv]
    n = len(sv)
    series = [np.ascontiguousarray(ALLTckResult(p).P_i, dtype=np.float64).ravel() for p in sv]
    stride = max(len(x) for x in series)
    P = np.zeros((n, stride))
    for i, x in enumerate(series):
        P[i, : len(x)] = x
    lens = np.array([len(x) for x in series], dtype=np.int64)
    eph = np.zeros((n, abi.EPH_NFIELDS, eph_cap))
    elen = np.zeros((n, abi.EPH_NFIELDS), dtype=np.int32)
    upd = np.zeros(n, dtype=np.int32)
    nav1 = np.zeros(n, dtype=np.int64)
    sfb1 = np.zeros(n, dtype=np.int64)
    o = abi.GnssNavOut()
    o.eph_cap = eph_cap
    o.eph = eph.ctypes.data_as(C.POINTER(C.c_double))
    o.eph_len = elen.ctypes.data_as(C.POINTER(C.c_int32))
    o.updateflag = upd.ctypes.data_as(C.POINTER(C.c_int32))
    o.nav1 = nav1.ctypes.data_as(C.POINTER(C.c_int64))
    o.sfb1 = sfb1.ctypes.data_as(C.POINTER(C.c_int64))
    a = to_c_acquired(Acquired)
    st = lib.gnss_navi_decode(C.byref(a), P.ctypes.data_as(C.POINTER(C.c_double)),
                              lens.ctypes.data_as(C.POINTER(C.c_int64)), stride, C.byref(o))
    if st != abi.OK:
        raise abi.GnssError(st, "gnss_navi_decode")
    entries = {}
    for i, p in enumerate(sv):
        e = SimpleNamespace(**{f: eph[i, k, : elen[i, k]].copy() for k, f in enumerate(abi.EPH_FIELDS)})
        e.updateflag = int(upd[i])
        entries[p] = e
    n1 = np.zeros(max(sv), dtype=np.int64)
    for i, p in enumerate(sv):
        n1[p - 1] = nav1[i]
    have = [p for i, p in enumerate(sv) if sfb1[i]]
    s1 = np.zeros(max(have) if have else 0, dtype=np.int64)
    for i, p in enumerate(sv):
        if sfb1[i]:
            s1[p - 1] = sfb1[i]
    for i, p in enumerate(sv):
        try:
            ALLTckResult(p).sfb1 = entries[p].sfb1.copy()
        except (AttributeError, TypeError):
            pass
    return StructArray(entries), ALLTckResult, SimpleNamespace(nav1=n1, sfb1=s1)


def colon(a: float, d: float, b: float) -> np.ndarray:
    """MATLAB's a:d:b with MathWorks' published colon construction (both ends toward the
    midpoint), the values the reference's tap vectors hold (e.g. -0.5:0.1:0.5 of the
    11-tap ACF, trackingCT_multiCorr-GIVEN.m:25). Same arithmetic as colon_make in
    csrc/gnss_internal.h."""
    if d == 0 or (a < b and d < 0) or (b < a and d > 0):
        return np.zeros(0)
    tol = 2.0 * 2.220446049250313e-16 * max(abs(a), abs(b))
    sig = 1.0 if d > 0 else -1.0
    if a == math.floor(a) and d == 1:
        n = math.floor(b) - a
    elif a == math.floor(a) and d == math.floor(d):
        q = math.floor(a / d)
        n = math.floor((b - (a - q * d)) / d) - q
    else:
        n = round((b - a) / d)  # (b - a)/d is never a half-integer for these ranges
        if sig * (a + n * d - b) > tol:
            n -= 1
    n = int(n)
    c = a + n * d
    if sig * (c - b) > -tol:
        c = b
    out = np.empty(n + 1)
    for k in range(n + 1):
        out[k] = (a + c) / 2 if 2 * k == n else (a + k * d if k <= n // 2 else c - (n - k) * d)
    return out


def ca_code(prn: int) -> np.ndarray:
    """generateCAcode(PRN) as used by the kernels (1023 chips of +-1)."""
    lib = abi.load()
    out = np.zeros(1023, dtype=np.int8)
    st = lib.gnss_ca_code(int(prn), out.ctypes.data_as(C.c_void_p))
    if st != abi.OK:
        raise abi.GnssError(st, "gnss_ca_code")
    return out


def vt_channel(prn, file_ptr, remChip, remCarrPhase, codeFreq, carrFreq, carrFreqBasis, oldCarrNco=0.0,
               oldCarrError=0.0):
    """A vector-tracking channel state (gnss_vt_chan): the initialisation of
    trackingVT_POS_updated.m:108-125 (from TckResultCT at msStartTckVT in the reference) and
    of the C/N0 estimator (:78-81: index_int 0, snrIndex 1)."""
    return abi.GnssVtChan(prn=int(prn), pad=0, file_ptr=int(file_ptr), remChip=float(remChip),
                          remCarrPhase=float(remCarrPhase), codeFreq=float(codeFreq), carrFreq=float(carrFreq),
                          carrFreqBasis=float(carrFreqBasis), oldCarrNco=float(oldCarrNco),
                          oldCarrError=float(oldCarrError), index_int=0, snrIndex=1)


def trackingVT_step(file, signal, track, chans, codeFreq_new, pdi=1, *, ctx: Context | None = None):
    """One step of trackingVT_POS_updated.m's tracking half (:157-349) for every channel on the
    GPU (gnss_tracking_vt_step): `chans` = a sequence of vt_channel states, advanced in place;
    codeFreq_new[i] = channel i's code frequency for this step, the caller's EKF prediction
    (:211-215). Returns one dict per channel: TckResultVT(prn).*(msIndex) (:319-346)."""
    ctx = ctx or default_context()
    n = len(chans)
    arr = (abi.GnssVtChan * n)(*chans)
    cf = np.ascontiguousarray(codeFreq_new, dtype=np.float64)
    if len(cf) != n:
        raise ValueError("one code frequency per channel")
    outs = (abi.GnssVtOut * n)()
    f, keep = to_c_file(file)
    s = to_c_signal(signal)
    t, keep2 = to_c_track(track)
    ctx.check(ctx.lib.gnss_tracking_vt_step(ctx.h, C.byref(f), C.byref(s), C.byref(t), int(pdi), n, arr,
                                            cf.ctypes.data_as(C.POINTER(C.c_double)), outs))
    for i in range(n):
        C.memmove(C.byref(chans[i]), C.byref(arr[i]), C.sizeof(abi.GnssVtChan))
    return [{k: (getattr(o, k)[:] if k == "sv_vel" else getattr(o, k)) for k, _ in abi.GnssVtOut._fields_}
            for o in outs]


def trackingVT_run(file, signal, track, chans, codeFreq_series, pdi=1, *, ctx: Context | None = None):
    """nsteps steps of trackingVT_POS_updated.m's tracking half (:157-349) for every channel in
    ONE launch (gnss_tracking_vt_run): codeFreq_series[s][i] = channel i's code frequency of
    step s (the caller's EKF prediction, :211-215, or a recorded series); `chans` advanced in
    place. Returns a dict of [nsteps][n] arrays: TckResultVT(prn).*(msIndex) (:319-346), CN0
    and cn0_row (CN0_VT(cn0_row, svindex), :301), status."""
    ctx = ctx or default_context()
    n = len(chans)
    cf = np.ascontiguousarray(codeFreq_series, dtype=np.float64)
    if cf.ndim != 2 or cf.shape[1] != n:
        raise ValueError("codeFreq_series: [nsteps][n]")
    nsteps = cf.shape[0]
    arr = (abi.GnssVtChan * n)(*chans)
    outs = (abi.GnssVtOut * (nsteps * n))()
    f, keep = to_c_file(file)
    s = to_c_signal(signal)
    t, keep2 = to_c_track(track)
    st = ctx.lib.gnss_tracking_vt_run(ctx.h, C.byref(f), C.byref(s), C.byref(t), int(pdi), n, nsteps, arr,
                                      cf.ctypes.data_as(C.POINTER(C.c_double)), outs)
    for i in range(n):
        C.memmove(C.byref(chans[i]), C.byref(arr[i]), C.sizeof(abi.GnssVtChan))
    rec = np.ctypeslib.as_array(outs).reshape(nsteps, n)  # a structured view of the records
    ctx.check(st)
    return {k: rec[k].copy() for k in rec.dtype.names}


def correlate_step(file, signal, prn, pdi, remChip, codeFreq, carrierFreq, remPhase, pos_bytes,
                   taps, *, ctx: Context | None = None):
    """One trackingCT correlation step on the GPU at an arbitrary NCO state
    (trackingCT.m:79-118 without negation / loop update). Returns (sums, numSample)
    with sums = [I_0, Q_0, I_1, Q_1, ...] per tap."""
    ctx = ctx or default_context()
    f, k1 = to_c_file(file)
    s = to_c_signal(signal)
    taps = np.ascontiguousarray(taps, dtype=np.float64)
    sums = np.zeros(2 * len(taps))
    ns = C.c_int64()
    ctx.check(ctx.lib.gnss_correlate_step(
        ctx.h, C.byref(f), C.byref(s), int(prn), int(pdi), float(remChip), float(codeFreq),
        float(carrierFreq), float(remPhase), int(pos_bytes), len(taps),
        taps.ctypes.data_as(C.POINTER(C.c_double)), sums.ctypes.data_as(C.POINTER(C.c_double)),
        C.byref(ns)))
    return sums, ns.value


# ---------------------------------------------------------------------------
# trackingVT_POS_updated.m: the EKF-driven vector-tracking loop
# ---------------------------------------------------------------------------
# global ALPHA BETA of initParameters.m:29-31 (the broadcast iono model, "From RINEX file")
ALPHA = [9.3132e-09, 1.4901e-08, -5.9605e-08, -1.1921e-07]
BETA = [8.8064e+04, 4.9152e+04, -1.3107e+05, -3.2768e+05]

VT_FIELDS = ["E_i", "E_q", "P_i", "P_q", "L_i", "L_q", "carrError", "codeError", "remChip", "remCarrPhase",
             "codeFreq", "carrFreq", "carrNco", "absoluteSample", "codedelay", "deltaPr", "prRate"]


def _struct_of(s, prn):
    """eph(prn) / TckResultCT(prn): a StructArray (or any callable), a dict keyed by PRN, or a
    sequence indexed like the MATLAB struct array (prn - 1)."""
    if callable(s):
        return s(prn)
    if isinstance(s, dict):
        return s[int(prn)]
    return s[int(prn) - 1]


def _first(x):
    return float(np.atleast_1d(np.asarray(x, dtype=np.float64)).ravel()[0])


def _vec1(v, prn):
    """sbf.nav1(prn): MATLAB 1-based vector indexing."""
    return _first(np.asarray(v).ravel()[int(prn) - 1])


def eph_sv(eph, prn, eph_idx=1):
    """The gnss_eph_sv of ephemeris(prn).*(eph_idx) (svPosVel.m:23-44; the VT loop passes
    eph_idx = 1, trackingVT_POS_updated.m:36)."""
    e = _struct_of(eph, prn)
    out = abi.GnssEphSv()
    for f in abi.EPH_SV_FIELDS:
        setattr(out, f, float(np.atleast_1d(np.asarray(getattr(e, f), dtype=np.float64)).ravel()[eph_idx - 1]))
    return out


def trackingVT_POS_updated(file, signal, track, cmn, solu, Acquired, cnslxyz, eph, sbf, TckResult_Eph,
                           TckResultCT, navSolutionsCT, *, ctx: Context | None = None, ALPHA_=None,
                           BETA_=None, nsteps: int | None = None, return_cn0: bool = False):
    """trackingVT_POS_updated.m:1-476 -> (TckResultVT, navSolutionsVT[, CN0_VT]).

    The loop of track.msToProcessVT / track.pdi steps: per step and channel the read size (:164)
    and the code frequency predicted from the EKF's receiver state (:180-227; host,
    gnss_vt_nav_predict), the E/P/L correlations, NCO, PLL and C/N0 of every channel in one
    GPU launch (:229-352), then the 8-state EKF on the code and carrier measurements
    (:357-467; host, gnss_vt_nav_update) -- all inside gnss_tracking_vt.

    Initialisation as the reference: the EKF state from navSolutionsCT row
    file.skiptimeVT / solu.navSolPeriod (:66-70), the channels from TckResultCT(prn) at
    msStartTckVT (:100-124: built from the LAST channel's sbf.nav1 / eph.sfb(1) and capped at
    that channel's record length, as the reference's loop variable leaves them),
    transmitTimeVT = navSolutionsCT.timeTransmit(1, :) (:131). TckResult_Eph only feeds
    sampleStart (:89-99), which no output reads; it is index-checked like MATLAB when given
    (the reference ships none: None skips the check). ALPHA_ / BETA_ default to
    initParameters.m's globals. nsteps overrides datalength / pdi (a shorter run).

    TckResultVT(prn) carries the fields of :324-352 (sv_vel as nsteps x 3; amplitude,
    navi_data, navi_dataL035 are the constant 0 the reference records); navSolutionsVT the
    rows of :418-436 (svxyz_pos n x 3 x nsteps, kalman_gain 8 x 2n x nsteps as the
    reference's 3-D arrays) and R (:466). A channel error MATLAB raises on (a replica index
    out of range, a read past the end of the record) raises GnssError.
    """
    ctx = ctx or default_context()
    sv = [int(p) for p in np.atleast_1d(Acquired.sv)]
    n = len(sv)
    if not 1 <= n <= abi.VT_MAX_CH:
        raise ValueError(f"vector tracking takes 1..{abi.VT_MAX_CH} channels")
    pdi = int(track.pdi)
    if nsteps is None:
        nsteps = int(track.msToProcessVT) // pdi
    row = file.skiptimeVT / solu.navSolPeriod
    if row != int(row) or row < 1:
        raise IndexError("file.skiptimeVT / solu.navSolPeriod must be a positive integer row (:66)")
    row = int(row)
    # :89-107
    if TckResult_Eph is not None:
        for p in sv:
            k = int(_vec1(sbf.nav1, p) + _first(_struct_of(eph, p).sfb) * 20)
            np.asarray(_struct_of(TckResult_Eph, p).absoluteSample).ravel()[k - 1]  # MATLAB's index check
    last = sv[-1]
    ms = int(_vec1(sbf.nav1, last) + _first(_struct_of(eph, last).sfb) * 20 + row)
    ms = min(ms, np.asarray(_struct_of(TckResultCT, last).codeFreq).size)
    chans = []
    for p in sv:  # :109-132
        t = _struct_of(TckResultCT, p)
        g = lambda f: float(np.asarray(getattr(t, f), dtype=np.float64).ravel()[ms - 1])
        c = vt_channel(p, int(g("absoluteSample")), g("remChip"), g("remCarrPhase"), g("codeFreq"),
                       g("carrFreq"), g("carrFreq"), g("carrFreq") - g("carrFreq"), g("carrError"))
        chans.append(c)
    arr = (abi.GnssVtChan * n)(*chans)
    cfg = abi.GnssVtNavCfg()
    cfg.cnslxyz[:] = [float(x) for x in np.asarray(cnslxyz, dtype=np.float64).ravel()[:3]]
    cfg.ALPHA[:] = [float(x) for x in (ALPHA_ if ALPHA_ is not None else ALPHA)]
    cfg.BETA[:] = [float(x) for x in (BETA_ if BETA_ is not None else BETA)]
    cfg.doy, cfg.cSpeed, cfg.Fc = float(cmn.doy), float(cmn.cSpeed), float(signal.Fc)
    ephs = (abi.GnssEphSv * n)(*[eph_sv(eph, p) for p in sv])
    ns = navSolutionsCT
    pos = (C.c_double * 3)(*np.asarray(ns.usrPos, dtype=np.float64)[row - 1, :3])
    vel = (C.c_double * 3)(*np.asarray(ns.usrVel, dtype=np.float64)[row - 1, :3])
    tt = (C.c_double * n)(*np.asarray(ns.timeTransmit, dtype=np.float64).reshape(-1, n)[0])
    s = to_c_signal(signal)
    nav = abi.GnssVtNav()
    st = ctx.lib.gnss_vt_nav_init(C.byref(cfg), C.byref(s), pdi, n, (C.c_int32 * n)(*sv), ephs, pos, vel,
                                  _vec1(ns.clkBias, row), _vec1(ns.clkDrift, row), tt, C.byref(nav))
    if st != abi.OK:
        raise abi.GnssError(st, "gnss_vt_nav_init")
    outs = (abi.GnssVtOut * (nsteps * n))()
    sols = (abi.GnssVtNavSol * nsteps)()
    f, keep = to_c_file(file)
    t, keep2 = to_c_track(track)
    st = ctx.lib.gnss_tracking_vt(ctx.h, C.byref(f), C.byref(s), C.byref(t), n, nsteps, arr, C.byref(nav), outs,
                                  sols)
    ctx.check(st)
    R = np.ctypeslib.as_array(outs).reshape(nsteps, n)  # a structured view of the records
    entries = {}
    for i, p in enumerate(sv):
        e = SimpleNamespace(**{k: R[k][:, i].astype(np.float64) for k in VT_FIELDS})
        e.sv_vel = R["sv_vel"][:, i].copy()
        for k in ("amplitude", "navi_data", "navi_dataL035"):
            setattr(e, k, np.zeros(nsteps))
        entries[p] = e
    nsol = _navsol_arrays(sols, nsteps, n)
    TckResultVT = StructArray(entries)
    if return_cn0:
        rows = int(R["cn0_row"].max()) if nsteps else 0
        cn0 = np.zeros((rows, n))
        for i in range(n):
            m = R["cn0_row"][:, i] > 0
            cn0[R["cn0_row"][:, i][m] - 1, i] = R["CN0"][:, i][m]
        return TckResultVT, nsol, cn0
    return TckResultVT, nsol


def _navsol_arrays(sols, nsteps, n):
    """navSolutionsVT (:418-436, :466) from the gnss_vt_navsol rows."""
    N = 2 * n
    S = np.ctypeslib.as_array(sols).reshape(nsteps)
    out = SimpleNamespace(**{k: S[k].copy() for k in ("localTime", "clkBias", "clkDrift")})
    for k in ("usrPos", "usrVel", "usrPosENU", "usrVelENU", "usrPosLLH", "satePos", "sateVel", "state",
              "state_cov"):
        setattr(out, k, S[k].copy())
    for k in ("meas_inno", "newZ", "predicted_z"):
        setattr(out, k, S[k][:, :N].copy())
    for k in ("satEA", "satAZ"):
        setattr(out, k, S[k][:, :n].copy())
    out.svxyz_pos = np.moveaxis(S["svxyz_pos"][:, :n], 0, -1).copy()          # n x 3 x nsteps
    out.kalman_gain = np.moveaxis(S["kalman_gain"][:, :, :N], 0, -1).copy()   # 8 x 2n x nsteps
    out.R = S["R"][S["r_row"] > 0][:, :N].copy()
    out.record_correction = np.zeros((nsteps, n))  # correction(svindex) = 0 (:128, :469)
    return out
