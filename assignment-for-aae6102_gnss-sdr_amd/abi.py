"""ctypes mirror of include/gnss_mi355x.h (the C-ABI drop-in boundary).

The struct layouts here must match the header field for field; tests check the
sizes against a tiny compiled probe. The product library is
``lib/libgnss_mi355x.so`` next to this file (built in-tree by
``__graft_entry__.build()``); if it is missing every entry point raises — there
is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

MAX_SV = 64
MAX_TAPS = 32

OK, ENODATA, EIO, EARG, EDEVICE, EINDEX = 0, 1, 2, 3, 4, 5

FIELDS = ["P_i", "P_q", "E_i", "E_q", "L_i", "L_q", "PLLdiscri", "DLLdiscri", "codedelay",
          "remChip", "codeFreq", "carrierFreq", "remPhase", "remSample", "numSample",
          "delayValue", "absoluteSample", "codedelay2"]
NFIELDS = len(FIELDS)
OUT_DEVICE = 1  # gnss_track_out.flags: rec / taps are device pointers (ABI v7)
# the same slots under trackingCT_POS_updated.m:273-292's names (gnss_tracking_ct_pos)
FIELDS_POS = ["P_i", "P_q", "E_i", "E_q", "L_i", "L_q", "carrError", "codeError", "codedelay",
              "remChip", "codeFreq", "carrFreq", "remCarrPhase", "absoluteSampleCodedelay",
              "numSample", "delayValue", "absoluteSample", "codedelay2"]

# the 25 taps of trackingCT_POS_updated_multicorrelator.m in Spacing order (0.6:-0.05:-0.6,
# :41), under the names of its TckResultCT fields (:374-423)
MC_TAPS = 25
MC_TAP_NAMES = ([f"E_{{}}{s}" for s in ["_060", "_055", "", "_045", "_040", "_035", "_030", "_025",
                                         "_020", "_015", "_010", "_005"]] + ["P_{}"] +
                [f"L_{{}}{s}" for s in ["005", "010", "015", "020", "025", "030", "035", "040", "045",
                                         "", "055", "060"]])


# ephemeris(prn) fields of naviDecode_updated.m (ini_eph.m order; updateflag separate)
EPH_FIELDS = ["TOW", "TOW1", "sfb", "sfb1", "weeknum", "N", "health", "IODC", "TGD", "toc", "af2",
              "af1", "af0", "IODE2", "Crs", "deltan", "M0", "Cuc", "ecc", "Cus", "sqrta", "toe", "Cic",
              "omegae", "Cis", "i0", "Crc", "w", "omegadot", "IODE3", "idot", "updatetime",
              "updatetime_tow"]
EPH_NFIELDS = len(EPH_FIELDS)


class GnssNavOut(C.Structure):
    _fields_ = [("eph_cap", C.c_int32), ("eph", C.POINTER(C.c_double)),
                ("eph_len", C.POINTER(C.c_int32)), ("updateflag", C.POINTER(C.c_int32)),
                ("nav1", C.POINTER(C.c_int64)), ("sfb1", C.POINTER(C.c_int64))]


class GnssFile(C.Structure):
    _fields_ = [("path", C.c_char_p), ("data", C.c_void_p), ("dev_data", C.c_void_p),
                ("nbytes", C.c_uint64), ("skip", C.c_int64), ("dataType", C.c_int32),
                ("dataPrecision", C.c_int32)]


class GnssSignal(C.Structure):
    _fields_ = [("IF", C.c_double), ("Fs", C.c_double), ("codeFreqBasis", C.c_double),
                ("ms", C.c_double), ("Sample", C.c_int64), ("codelength", C.c_double)]


class GnssAcq(C.Structure):
    _fields_ = [("freqNum", C.c_int32), ("freqMin", C.c_double), ("freqStep", C.c_double),
                ("datalen", C.c_int32), ("L", C.c_int32), ("n_prn", C.c_int32),
                ("prn_list", C.POINTER(C.c_int32))]


class GnssAcquired(C.Structure):
    _fields_ = [("n", C.c_int32), ("sv", C.c_int32 * MAX_SV), ("SNR", C.c_double * MAX_SV),
                ("Doppler", C.c_double * MAX_SV), ("codedelay", C.c_int32 * MAX_SV),
                ("fineFreq", C.c_double * MAX_SV)]


class GnssAcqDiag(C.Structure):
    _fields_ = [("n", C.c_int32), ("prn", C.c_int32 * MAX_SV), ("SNR", C.c_double * MAX_SV),
                ("fbin", C.c_int32 * MAX_SV), ("codePhase", C.c_int32 * MAX_SV),
                ("peak", C.c_double * MAX_SV), ("peak2", C.c_double * MAX_SV)]


class GnssTrack(C.Structure):
    _fields_ = [("CorrelatorSpacing", C.c_double), ("DLLBW", C.c_double), ("DLLDamp", C.c_double),
                ("DLLGain", C.c_double), ("PLLBW", C.c_double), ("PLLDamp", C.c_double),
                ("PLLGain", C.c_double), ("msToProcessCT_1ms", C.c_int32),
                ("msToProcessCT_10ms", C.c_int32), ("n_taps", C.c_int32),
                ("tap_offsets", C.POINTER(C.c_double)), ("n_chan", C.c_int32),
                ("chan", C.POINTER(C.c_int32))]


class GnssTrackOut(C.Structure):
    _fields_ = [("max_len", C.c_int64), ("rec", C.POINTER(C.c_double)),
                ("taps", C.POINTER(C.c_double)), ("len", C.POINTER(C.c_int64)),
                ("countinx", C.POINTER(C.c_int32)), ("CN0_Eph", C.POINTER(C.c_double)),
                ("cn0_cap", C.c_int32), ("cn0_rows", C.c_int32), ("flags", C.c_int32),
                ("reserved", C.c_int32)]


class GnssTiming(C.Structure):
    _fields_ = [("acq_ms", C.c_double), ("acq_corr_ms", C.c_double), ("acq_fine_ms", C.c_double),
                ("track_ms", C.c_double), ("track_kernel_ms", C.c_double),
                ("track_launches", C.c_int64), ("track_channel_samples", C.c_int64),
                ("acq_hypothesis_samples", C.c_int64), ("h2d_ms", C.c_double),
                ("track10_kernel_ms", C.c_double), ("track10_launches", C.c_int64),
                ("track10_channel_samples", C.c_int64), ("h2d_bytes", C.c_int64),
                ("track_segments", C.c_int64)]


class GnssVtChan(C.Structure):
    _fields_ = [("prn", C.c_int32), ("pad", C.c_int32), ("file_ptr", C.c_int64), ("remChip", C.c_double),
                ("remCarrPhase", C.c_double), ("codeFreq", C.c_double), ("carrFreq", C.c_double),
                ("carrFreqBasis", C.c_double), ("oldCarrNco", C.c_double), ("oldCarrError", C.c_double),
                ("index_int", C.c_int32), ("snrIndex", C.c_int32), ("Zk", C.c_double * 20)]


class GnssVtOut(C.Structure):
    _fields_ = [(f, C.c_double) for f in ("E_i", "E_q", "P_i", "P_q", "L_i", "L_q", "carrError", "codeError",
                                          "carrNco", "remChip", "remCarrPhase", "codeFreq", "carrFreq")] + \
               [("numSample", C.c_int64), ("absoluteSample", C.c_int64), ("codedelay", C.c_double),
                ("CN0", C.c_double), ("cn0_row", C.c_int32), ("status", C.c_int32),
                ("deltaPr", C.c_double), ("prRate", C.c_double), ("sv_vel", C.c_double * 3)]


# the vector half of trackingVT_POS_updated.m (ABI v10)
VT_MAX_CH = 32
EPH_SV_FIELDS = ["sqrta", "deltan", "toe", "M0", "ecc", "w", "Cus", "Cuc", "Crs", "Crc", "Cis", "Cic", "i0",
                 "idot", "omegae", "omegadot", "toc", "af0", "af1", "af2", "TGD"]
GEO_XYZ2LLH, GEO_LLH2XYZ, GEO_XYZ2ENU, GEO_EROTCORR, GEO_IONO, GEO_TROP = range(6)


class GnssEphSv(C.Structure):
    _fields_ = [(f, C.c_double) for f in EPH_SV_FIELDS]


class GnssVtNavCfg(C.Structure):
    _fields_ = [("cnslxyz", C.c_double * 3), ("ALPHA", C.c_double * 4), ("BETA", C.c_double * 4),
                ("doy", C.c_double), ("cSpeed", C.c_double), ("Fc", C.c_double)]


class GnssVtNav(C.Structure):
    _fields_ = [("n", C.c_int32), ("pdi", C.c_int32), ("msIndex", C.c_int32), ("counterUptR", C.c_int32),
                ("counter_r", C.c_int32), ("prn", C.c_int32 * VT_MAX_CH), ("cfg", GnssVtNavCfg),
                ("Fs", C.c_double), ("IF", C.c_double), ("codeFreqBasis", C.c_double), ("ms", C.c_double),
                ("cnslxyz", C.c_double * 3), ("total_state", C.c_double * 8), ("state_cov", C.c_double * 64),
                ("R", C.c_double * (2 * VT_MAX_CH)), ("recordR2", C.c_double * (2 * VT_MAX_CH))] + \
               [(f, C.c_double * VT_MAX_CH) for f in ("transmitTime", "tot_est_tck", "predictedPr_last",
                                                     "counter_corr", "ionodel", "tropodel", "el", "az")] + \
               [("numSample", C.c_int64 * VT_MAX_CH), ("eph", GnssEphSv * VT_MAX_CH)]


class GnssVtNavSol(C.Structure):
    _fields_ = [("localTime", C.c_double)] + \
               [(f, C.c_double * 3) for f in ("usrPos", "usrVel", "usrPosENU", "usrVelENU", "usrPosLLH")] + \
               [("clkBias", C.c_double), ("clkDrift", C.c_double), ("state", C.c_double * 8),
                ("state_cov", C.c_double * 8), ("newZ", C.c_double * (2 * VT_MAX_CH)),
                ("meas_inno", C.c_double * (2 * VT_MAX_CH)), ("satEA", C.c_double * VT_MAX_CH),
                ("satAZ", C.c_double * VT_MAX_CH), ("predicted_z", C.c_double * (2 * VT_MAX_CH)),
                ("satePos", C.c_double * 3), ("sateVel", C.c_double * 3),
                ("svxyz_pos", (C.c_double * 3) * VT_MAX_CH), ("kalman_gain", (C.c_double * (2 * VT_MAX_CH)) * 8),
                ("R", C.c_double * (2 * VT_MAX_CH)), ("r_row", C.c_int32),
                ("reserved", C.c_int32)]


class GnssSynthSv(C.Structure):
    _fields_ = [("prn", C.c_int32), ("doppler_hz", C.c_double), ("code_phase0", C.c_double),
                ("carr_phase0", C.c_double), ("cn0_dbhz", C.c_double), ("bit_seed", C.c_uint64),
                ("bit_phase_chips", C.c_double), ("lnav", C.c_int32), ("reserved", C.c_int32)]


class GnssSynth(C.Structure):
    _fields_ = [("Fs", C.c_double), ("IF", C.c_double), ("noise_sigma", C.c_double),
                ("seed", C.c_uint64), ("n_sv", C.c_int32), ("sv", GnssSynthSv * MAX_SV)]


# exported symbols and their prototypes (checked by tests against the header)
PROTOTYPES = {
    "gnss_abi_version": (C.c_int, []),
    "gnss_strerror": (C.c_char_p, [C.c_int]),
    "gnss_ctx_create": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "gnss_ctx_create_multi": (C.c_int, [C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_void_p)]),
    "gnss_ctx_members": (C.c_int, [C.c_void_p]),
    "gnss_ctx_drop_record": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gnss_ctx_resident_records": (C.c_int, [C.c_void_p]),
    "gnss_device_count": (C.c_int, []),
    "gnss_ctx_destroy": (None, [C.c_void_p]),
    "gnss_last_error": (C.c_char_p, [C.c_void_p]),
    "gnss_last_timing": (C.c_int, [C.c_void_p, C.POINTER(GnssTiming)]),
    "gnss_ctx_set_profiling": (C.c_int, [C.c_void_p, C.c_int]),
    "gnss_ctx_set_acq_precision": (C.c_int, [C.c_void_p, C.c_int]),
    "gnss_ctx_set_window": (C.c_int, [C.c_void_p, C.c_uint64]),
    "gnss_ctx_set_option": (C.c_int, [C.c_void_p, C.c_int, C.c_int64]),
    "gnss_dev_alloc": (C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(C.c_void_p)]),
    "gnss_dev_free": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gnss_dev_upload": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]),
    "gnss_dev_download": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]),
    "gnss_acquisition": (C.c_int, [C.c_void_p, C.POINTER(GnssFile), C.POINTER(GnssSignal),
                                   C.POINTER(GnssAcq), C.POINTER(GnssAcquired),
                                   C.POINTER(GnssAcqDiag)]),
    "gnss_tracking_ct": (C.c_int, [C.c_void_p, C.POINTER(GnssFile), C.POINTER(GnssSignal),
                                   C.POINTER(GnssTrack), C.POINTER(GnssAcquired),
                                   C.POINTER(GnssTrackOut)]),
    "gnss_tracking_ct_pos": (C.c_int, [C.c_void_p, C.POINTER(GnssFile), C.POINTER(GnssSignal),
                                       C.POINTER(GnssTrack), C.POINTER(GnssAcquired), C.c_int32,
                                       C.POINTER(C.c_int32), C.POINTER(GnssTrackOut)]),
    "gnss_tracking_ct_mc": (C.c_int, [C.c_void_p, C.POINTER(GnssFile), C.POINTER(GnssSignal),
                                      C.POINTER(GnssTrack), C.POINTER(GnssAcquired), C.c_int32,
                                      C.c_int32, C.POINTER(GnssTrackOut)]),
    "gnss_tracking_ct_multicorr": (C.c_int, [C.c_void_p, C.POINTER(GnssFile), C.POINTER(GnssSignal),
                                             C.POINTER(GnssTrack), C.POINTER(GnssAcquired), C.c_int32,
                                             C.POINTER(GnssTrackOut)]),
    "gnss_navi_decode": (C.c_int, [C.POINTER(GnssAcquired), C.POINTER(C.c_double),
                                   C.POINTER(C.c_int64), C.c_int64, C.POINTER(GnssNavOut)]),
    "gnss_lnav_bits": (C.c_int, [C.c_int32, C.c_int32, C.c_void_p]),
    "gnss_ca_code": (C.c_int, [C.c_int, C.c_void_p]),
    "gnss_correlate_step": (C.c_int, [C.c_void_p, C.POINTER(GnssFile), C.POINTER(GnssSignal),
                                      C.c_int, C.c_int, C.c_double, C.c_double, C.c_double,
                                      C.c_double, C.c_int64, C.c_int, C.POINTER(C.c_double),
                                      C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
    "gnss_synth_if_device": (C.c_int, [C.c_void_p, C.POINTER(GnssSynth), C.c_uint64, C.c_uint64,
                                       C.c_void_p]),
    "gnss_tracking_vt_run": (C.c_int, [C.c_void_p, C.POINTER(GnssFile), C.POINTER(GnssSignal),
                                       C.POINTER(GnssTrack), C.c_int32, C.c_int32, C.c_int32,
                                       C.POINTER(GnssVtChan), C.POINTER(C.c_double), C.POINTER(GnssVtOut)]),
    "gnss_tracking_vt_step": (C.c_int, [C.c_void_p, C.POINTER(GnssFile), C.POINTER(GnssSignal),
                                        C.POINTER(GnssTrack), C.c_int32, C.c_int32, C.POINTER(GnssVtChan),
                                        C.POINTER(C.c_double), C.POINTER(GnssVtOut)]),
    "gnss_vt_nco_step": (C.c_int, [C.POINTER(GnssSignal), C.POINTER(GnssTrack), C.c_int32,
                                   C.POINTER(GnssVtChan), C.c_double, C.c_double, C.c_double,
                                   C.POINTER(GnssVtOut)]),
    "gnss_vt_prepare": (C.c_int, [C.POINTER(GnssSignal), C.c_int32, C.POINTER(GnssVtChan), C.c_double,
                                  C.POINTER(C.c_int32), C.POINTER(C.c_int64)]),
    "gnss_sv_pos_vel": (C.c_int, [C.POINTER(GnssEphSv), C.c_double, C.POINTER(C.c_double),
                                  C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double),
                                  C.POINTER(C.c_double)]),
    "gnss_geo": (C.c_int, [C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "gnss_vt_nav_init": (C.c_int, [C.POINTER(GnssVtNavCfg), C.POINTER(GnssSignal), C.c_int32, C.c_int32,
                                   C.POINTER(C.c_int32), C.POINTER(GnssEphSv), C.POINTER(C.c_double),
                                   C.POINTER(C.c_double), C.c_double, C.c_double, C.POINTER(C.c_double),
                                   C.POINTER(GnssVtNav)]),
    "gnss_vt_nav_predict": (C.c_int, [C.POINTER(GnssVtNav), C.c_int32, C.c_int64, C.POINTER(C.c_double),
                                      C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "gnss_vt_nav_update": (C.c_int, [C.POINTER(GnssVtNav), C.POINTER(C.c_double), C.POINTER(C.c_double),
                                     C.POINTER(C.c_double), C.POINTER(GnssVtNavSol)]),
    "gnss_tracking_vt": (C.c_int, [C.c_void_p, C.POINTER(GnssFile), C.POINTER(GnssSignal), C.POINTER(GnssTrack),
                                   C.c_int32, C.c_int32, C.POINTER(GnssVtChan), C.POINTER(GnssVtNav),
                                   C.POINTER(GnssVtOut), C.POINTER(GnssVtNavSol)]),
}

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libgnss_mi355x.so")
_lib = None
_torch_first = False
LOADED_PATH = None  # the library file the process bound (bench.py digests it)

# gnss_ctx_set_option keys (include/gnss_mi355x.h, ABI v11)
(OPT_FORCE_SUB, OPT_NO_PERSIST, OPT_FORCE_VPB, OPT_ACQ_ROCFFT, OPT_FINE_ROCFFT, OPT_ACQ_BATCH, OPT_ACQ_FUSED,
 OPT_ACQ_RING, OPT_ACQ_PIPE, OPT_VT_BLOCKS, OPT_FORCE_PEER, OPT_VT_SPAN) = range(12)
MAX_DEVICES = 16


def require_torch():
    """torch, for the entry points that exchange device tensors with the library; raises if
    the library was loaded before torch (torch would then see no GPU in this process)."""
    import torch
    if _lib is not None and not _torch_first:
        raise RuntimeError("import torch before the first gnss Context / abi.load() "
                           "(PyTorch-ROCm must bring up its HIP runtime first)")
    return torch


class GnssError(RuntimeError):
    def __init__(self, status, msg=""):
        self.status = status
        super().__init__(f"gnss status {status}: {msg}")


def load(path: str | None = None):
    """Load the HIP C-ABI library (raises if it has not been built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # GNSS_LIB: a timing-probe build (tools/build_probe.sh) in place of the product library
    p = path or os.environ.get("GNSS_LIB") or LIB_PATH
    if not os.path.exists(p):
        raise ImportError(f"{p} missing: the HIP extension is not built "
                          "(run `python -c 'import __graft_entry__ as g; g.build()'`)")
    # PyTorch-ROCm ships its own HIP / HSA runtime and finds no GPU if this library's runtime
    # came up first, so it is imported here, before the library, whenever it is installed: a
    # caller may create a Context first and hand tensors over later (device-resident outputs,
    # the RCCL gathers). require_torch() still checks the order for a library loaded without
    # torch installed at the time.
    global _torch_first
    if _lib is None:
        if "torch" not in sys.modules and os.environ.get("GNSS_NO_TORCH", "0") != "1":
            try:  # PyTorch's runtime first: any later tensor exchange then works
                import torch  # noqa: F401
            except Exception:  # (a torch that fails to import, e.g. an OSError from its ROCm
                pass  # libraries, must not stop the GNSS library from loading; require_torch() checks)
        _torch_first = "torch" in sys.modules
    lib = C.CDLL(p)
    for name, (res, args) in PROTOTYPES.items():
        if p != LIB_PATH and not hasattr(lib, name):
            continue  # (an A/B or probe build of another revision: entry points it lacks stay unbound)
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        global LOADED_PATH
        _lib = lib
        LOADED_PATH = os.path.abspath(p)
    return lib
