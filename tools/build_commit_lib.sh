# A/B builds: the library (probe build: GNSS_PROBE_BUILD=1, the GNSS_STAMPS hook on) as it was
# at each given commit, into tools/probe_lib/libgnss_<commit>.so (git worktree in /tmp).
# Load one with GNSS_LIB=<path> (abi.load skips entry points an older library lacks).
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
mkdir -p "$ROOT/tools/probe_lib"
for c in "$@"; do
  W=/tmp/gnss_wt_$c
  rm -rf "$W"; git -C "$ROOT" worktree prune
  git -C "$ROOT" worktree add -f --detach "$W" "$c" >/dev/null
  (cd "$W/assignment-for-aae6102_gnss-sdr_amd/csrc" && make -s FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -pthread -Wall -Wno-unused-function -DGNSS_PROBE_BUILD=1" >/dev/null 2>&1)
  cp "$W/assignment-for-aae6102_gnss-sdr_amd/lib/libgnss_mi355x.so" "$ROOT/tools/probe_lib/libgnss_$c.so"
  git -C "$ROOT" worktree remove --force "$W"
  echo "built tools/probe_lib/libgnss_$c.so"
done
