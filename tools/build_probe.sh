# Timing-probe variants of the library (GNSS_CORR_PROBE bits, track.hip): builds
# tools/probe_lib/libgnss_probe<N>.so for each N given; load one with GNSS_LIB=<path>.
# Never used by the product, the tests or bench.py.
set -e
cd "$(dirname "$0")/../assignment-for-aae6102_gnss-sdr_amd/csrc"
make -s
mkdir -p ../../tools/probe_lib /tmp/gnss_probe_obj
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -pthread"
for n in "$@"; do
  /opt/rocm/bin/hipcc $FLAGS -DGNSS_CORR_PROBE=$n -c track.hip -o /tmp/gnss_probe_obj/track_$n.o &
done
wait
for n in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/probe_lib/libgnss_probe$n.so \
    /tmp/gnss_probe_obj/track_$n.o ../build/acq.o ../build/acq_fft.o ../build/synth.o ../build/ifmt.o \
    ../build/gnss_api.o -L/opt/rocm/lib -lrocfft -pthread -Wl,-rpath,/opt/rocm/lib
done
ls -la ../../tools/probe_lib
