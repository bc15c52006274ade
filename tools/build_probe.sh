# Timing-probe variants of the library: builds tools/probe_lib/libgnss_probe<N>.so for each
# N given, with GNSS_CORR_PROBE=N (track.hip: bits that drop parts of the correlator; 0 =
# the full correlator) and GNSS_PROBE_BUILD=1 (gnss_api.cpp reads the GNSS_STAMPS /
# GNSS_PROBE / GNSS_HOSTPROF / GNSS_FORCE_SUB10 environment hooks). Load one with
# GNSS_LIB=<path>. Never used by the product, the tests or bench.py. EXTRA_FLAGS adds
# compiler flags (e.g. -DGNSS_XCHG_LD_POL=17: the exchange's poll cache policy).
set -e
cd "$(dirname "$0")/../assignment-for-aae6102_gnss-sdr_amd/csrc"
make -s
mkdir -p ../../tools/probe_lib /tmp/gnss_probe_obj
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -pthread -DGNSS_PROBE_BUILD=1 $EXTRA_FLAGS"
/opt/rocm/bin/hipcc $FLAGS -c gnss_api.cpp -o /tmp/gnss_probe_obj/gnss_api.o &
for n in "$@"; do
  /opt/rocm/bin/hipcc $FLAGS -DGNSS_CORR_PROBE=$n -c track.hip -o /tmp/gnss_probe_obj/track_$n.o &
done
wait
for n in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/probe_lib/libgnss_probe$n.so \
    /tmp/gnss_probe_obj/track_$n.o /tmp/gnss_probe_obj/gnss_api.o \
    $(ls ../build/*.o | grep -v -e '/track.o$' -e '/gnss_api.o$') \
    -L/opt/rocm/lib -lrocfft -pthread -Wl,-rpath,/opt/rocm/lib
done
ls -la ../../tools/probe_lib
