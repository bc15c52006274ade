# Product-flag variants of the library for A/B runs: `[SRC=vt] bash tools/build_variant.sh NAME -DKNOB=v ...`
# compiles track.hip (or $SRC.hip) with the extra flags, links it with the product's other objects
# (../build/*.o, `make` first) into tools/probe_lib/libgnss_NAME.so. Load with GNSS_LIB=<path>
# (tools/gpu.sh ab). Never used by the product, the tests or bench.py.
set -e
cd "$(dirname "$0")/../assignment-for-aae6102_gnss-sdr_amd/csrc"
make -s
mkdir -p ../../tools/probe_lib /tmp/gnss_variant_obj
NAME=$1; shift
SRC=${SRC:-track}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -pthread -Wall -Wno-unused-function "$@" \
  -c $SRC.hip -o /tmp/gnss_variant_obj/${SRC}_$NAME.o
OBJS=$(ls ../build/*.o | grep -v "/$SRC.o$")
if [ -n "$PROBE" ]; then  # PROBE=1: the host side's probe hooks too (GNSS_STAMPS, GNSS_PROBE environment)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -pthread -DGNSS_PROBE_BUILD=1 \
    -c gnss_api.cpp -o /tmp/gnss_variant_obj/gnss_api_$NAME.o
  OBJS="$(echo $OBJS | tr ' ' '\n' | grep -v '/gnss_api.o$' | tr '\n' ' ') /tmp/gnss_variant_obj/gnss_api_$NAME.o"
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/probe_lib/libgnss_$NAME.so \
  /tmp/gnss_variant_obj/${SRC}_$NAME.o $OBJS -L/opt/rocm/lib -lrocfft -pthread -Wl,-rpath,/opt/rocm/lib
echo "built tools/probe_lib/libgnss_$NAME.so"
