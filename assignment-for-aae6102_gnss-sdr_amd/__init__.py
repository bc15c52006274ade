"""MI355X-native GPS L1 C/A acquisition + conventional tracking (drop-in for
acquisition.m / trackingCT.m of KangWelly/Assignment-for-AAE6102_GNSS-SDR, plus the tracking
loops of trackingCT_POS_updated.m and trackingCT_POS_updated_multicorrelator.m and
naviDecode_updated.m).

The compute path is the HIP C-ABI library lib/libgnss_mi355x.so (hand-written
gfx950 kernels); this package is the host-side mirror of the
reference's MATLAB interface. Import with
``importlib.import_module("assignment-for-aae6102_gnss-sdr_amd")`` (the
directory name is not a Python identifier).
"""
from . import abi, synth
from .sdr import (Context, DeviceRecord, DeviceTrackOutBuffers, StructArray, TrackOutBuffers, acquisition, ca_code, colon,
                  default_context, initParameters, naviDecode_updated, trackingCT, trackingCT_multiCorr,
                  trackingCT_POS, trackingCT_POS_updated_multicorrelator, trackingVT_POS_updated, trackingVT_run, trackingVT_step,
                  vt_channel)

__all__ = ["abi", "synth", "Context", "DeviceRecord", "DeviceTrackOutBuffers", "StructArray", "TrackOutBuffers",
           "acquisition", "ca_code", "colon", "default_context", "initParameters", "naviDecode_updated",
           "trackingCT", "trackingCT_multiCorr", "trackingCT_POS", "trackingCT_POS_updated_multicorrelator", "trackingVT_POS_updated", "trackingVT_run", "trackingVT_step",
           "vt_channel"]
