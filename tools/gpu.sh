# One MI355X check, run from the repo root via gpurun:
#   gpurun --timeout 1200 -- bash tools/gpu.sh STEP [STEP ...]
# Steps run in order, each under its own time limit; the first failure ends the call.
#   tests        pytest -m gpu (PYTEST_K="expr" narrows it to -k expr)
#   bench        python bench.py (BENCH_ARGS adds flags) -> gpurun_out/bench.json
#   prof         rocprofv3 --kernel-trace --stats of one bench step -> gpurun_out/prof_bench(_summary.txt)
#   traffic      FETCH_SIZE / WRITE_SIZE passes of the 10-ms tracking launch -> gpurun_out/traffic.json
#   tracksq      SQ counter passes (VALU / LDS / waits) of the tracking launches -> gpurun_out/track_sq.json
#   acqpmc       FETCH / WRITE + SQ passes of the fp64 acquisition kernels -> gpurun_out/acq_counters.json
#   probes       per timing-probe library (PROBES="0 1 2 8"): SQ fp64/VALU counts and GNSS_STAMPS
#   probes1      the same libraries' GNSS_STAMPS of the 1-ms phase alone (tools/track_only.py 1000 0)
#   acqab        rocprofv3 kernel stats of the config-2 acquisition: two-launch path, then the
#                fused correlator at ring depths $RINGS (default "3"); + its FETCH/WRITE bytes
#   acqpmc4      FETCH / WRITE passes of the config-4 acquisition's correlator kernels -> gpurun_out/traffic_cfg4.json
#   acqprof1     kernel stats of the config-2 acquisition, passes on one stream -> gpurun_out/acq_onestream_summary.txt
#   acqpipe      config-2 / config-4 acquisition timing, batches on one stream vs pipelined (tools/acq_only.py)
#   spawn        bench.py --gpus 2 without a launcher (own ranks, gloo, one device)
#   cfg4         bench --workload cfg4 -> gpurun_out/bench_cfg4.json
#   cfg5         bench --workload cfg5 -> gpurun_out/bench_cfg5.json
#   vt           tools/vt_only.py: the VT loop's wall / kernel time per step -> gpurun_out/vt_only.txt
#   cfg5pmc      the config-5 launch's PMC traffic + SQ passes -> gpurun_out/{traffic_cfg5,cfg5_sq}.json
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd "$R" || exit 1
SQ1="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
SQ2="SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA"
SQ3="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU"
pmc() {  # pmc OUTDIR "COUNTERS" cmd...
  local out=$1 ctrs=$2; shift 2
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d "$R/gpurun_out/$out" -o run -- "$@" ) > "gpurun_out/$out.log" 2>&1 || { tail -20 "gpurun_out/$out.log"; return 1; }
}
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    tests)
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1 \
        && echo "TESTS_OK $(tail -1 gpurun_out/pytest_gpu.log)" || { grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | tail -30; tail -40 gpurun_out/pytest_gpu.log; exit 1; } ;;
    bench)
      timeout -k 10 400 python3 bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err \
        && tail -1 gpurun_out/bench.json | cut -c1-700 || { tail -20 gpurun_out/bench.err; exit 1; } ;;
    prof)
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_bench" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu ) > gpurun_out/bench_prof.json 2>&1 || { tail -20 gpurun_out/bench_prof.json; exit 1; }
      python3 tools/prof_summary.py gpurun_out/prof_bench > gpurun_out/prof_bench_summary.txt && head -14 gpurun_out/prof_bench_summary.txt ;;
    traffic)
      pmc pmc_fetch FETCH_SIZE python3 "$R/tools/track_only.py" 1000 40000 || exit 1
      pmc pmc_write WRITE_SIZE python3 "$R/tools/track_only.py" 1000 40000 || exit 1
      python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write "track_run_kernel<3, 3, false, false>" gpurun_out/traffic.json || exit 1
      rm -f gpurun_out/pmc_*/**/*kernel_trace.csv ;;
    tracksq)
      pmc trk_sq1 "$SQ1" python3 "$R/tools/track_only.py" 1000 400 || exit 1
      pmc trk_sq2 "$SQ2" python3 "$R/tools/track_only.py" 1000 400 || exit 1
      pmc trk_sq3 "$SQ3" python3 "$R/tools/track_only.py" 1000 400 || exit 1
      python3 tools/pmc_sq.py gpurun_out/track_sq.json gpurun_out/trk_sq1 gpurun_out/trk_sq2 gpurun_out/trk_sq3 -- "track_run_kernel<3, 3, false, false>" "track_run_kernel<3, 1, false, false>" || exit 1
      rm -f gpurun_out/trk_sq*/**/*kernel_trace.csv ;;
    acqpmc)
      pmc acq_fetch FETCH_SIZE python3 "$R/tools/acq_only.py" || exit 1
      pmc acq_write WRITE_SIZE python3 "$R/tools/acq_only.py" || exit 1
      pmc acq_sq1 "$SQ1" python3 "$R/tools/acq_only.py" || exit 1
      pmc acq_sq2 "$SQ2" python3 "$R/tools/acq_only.py" || exit 1
      python3 tools/pmc_sq.py gpurun_out/acq_counters.json gpurun_out/acq_fetch gpurun_out/acq_write gpurun_out/acq_sq1 gpurun_out/acq_sq2 -- "inv_cols_kernel<29, HIP_vector_type<double" "inv_rows_kernel_f64<29>" "fwd_rows_kernel<29" "fine_rows_kernel<29" "fine_cols_kernel<29>" || exit 1
      rm -f gpurun_out/acq_*/**/*kernel_trace.csv ;;
    acqab)
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/acqab_split" -o run -- python3 "$R/tools/acq_only.py" ) > gpurun_out/acqab_split.log 2>&1 || { tail -20 gpurun_out/acqab_split.log; exit 1; }
      python3 tools/prof_summary.py gpurun_out/acqab_split | head -6
      for r in ${RINGS:-3}; do
        ( cd /tmp && export TMPDIR=/tmp && ACQ_FUSED=$r timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/acqab_f$r" -o run -- python3 "$R/tools/acq_only.py" ) > gpurun_out/acqab_f$r.log 2>&1 || { tail -20 gpurun_out/acqab_f$r.log; exit 1; }
        echo "ring $r:"; python3 tools/prof_summary.py gpurun_out/acqab_f$r | head -4
      done
      ACQ_FUSED=3 pmc acqf_fetch FETCH_SIZE python3 "$R/tools/acq_only.py" || exit 1
      ACQ_FUSED=3 pmc acqf_write WRITE_SIZE python3 "$R/tools/acq_only.py" || exit 1
      python3 tools/pmc_sq.py gpurun_out/acq_fused_bytes.json gpurun_out/acqf_fetch gpurun_out/acqf_write -- "inv_fused_kernel_f64<29>" || exit 1
      rm -f gpurun_out/acq*/**/*kernel_trace.csv ;;
    acqpmc4)
      ACQ_CFG=4 pmc a4_fetch FETCH_SIZE python3 "$R/tools/acq_only.py" || exit 1
      ACQ_CFG=4 pmc a4_write WRITE_SIZE python3 "$R/tools/acq_only.py" || exit 1
      python3 tools/pmc_call_bytes.py gpurun_out/a4_fetch gpurun_out/a4_write 3 gpurun_out/traffic_cfg4.json \
        "tools/acq_only.py with ACQ_CFG=4 (the bench's config-4 record, 32 PRNs x 81 bins x 10 ms, fp64), the correlator's kernels (forward rows/cols, inverse cols/rows)" \
        "fwd_rows_kernel<13" "fwd_cols_kernel<13" "inv_cols_kernel<13" "inv_rows_kernel_f64<13>" || exit 1
      rm -f gpurun_out/a4_*/**/*kernel_trace.csv ;;
    spawn)  # bench.py --gpus 2 with no launcher: its own two ranks, both on device 0 over gloo (the
      # one-GPU rehearsal of the driver's `python3 bench.py --gpus N`; SPAWN_WL = workload)
      BENCH_FORCE_DEVICE=0 BENCH_DIST_BACKEND=gloo timeout -k 10 500 python3 bench.py --gpus 2 --workload ${SPAWN_WL:-cfg2+3} --steps 2 --warmup 1 --no-cpu --no-profile-pass $BENCH_ARGS > gpurun_out/bench_spawn.json 2> gpurun_out/bench_spawn.err \
        && tail -1 gpurun_out/bench_spawn.json | cut -c1-900 || { tail -20 gpurun_out/bench_spawn.err; exit 1; } ;;
    multictx)  # the headline through the C-ABI multi-device context in one process (MULTI_DEVICES, default 0,0
      # on the one-GPU box: two members on device 0, one after the other)
      BENCH_MULTI_DEVICES=${MULTI_DEVICES:-0,0} timeout -k 10 500 python3 bench.py --multi-ctx 2 --steps 3 --warmup 1 $BENCH_ARGS > gpurun_out/bench_multictx.json 2> gpurun_out/bench_multictx.err \
        && tail -1 gpurun_out/bench_multictx.json | cut -c1-1200 || { tail -20 gpurun_out/bench_multictx.err; exit 1; } ;;
    cfg4)
      timeout -k 10 400 python3 bench.py --workload cfg4 $BENCH_ARGS > gpurun_out/bench_cfg4.json 2> gpurun_out/bench_cfg4.err \
        && tail -1 gpurun_out/bench_cfg4.json | cut -c1-500 || { tail -20 gpurun_out/bench_cfg4.err; exit 1; } ;;
    cfg5)
      timeout -k 10 500 python3 bench.py --workload cfg5 $BENCH_ARGS > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err \
        && tail -1 gpurun_out/bench_cfg5.json | cut -c1-700 || { tail -20 gpurun_out/bench_cfg5.err; exit 1; } ;;
    cfg5pmc)
      pmc c5_fetch FETCH_SIZE python3 "$R/tools/track_only.py" 1000 90000 11 32 || exit 1
      pmc c5_write WRITE_SIZE python3 "$R/tools/track_only.py" 1000 90000 11 32 || exit 1
      python3 tools/pmc_traffic.py gpurun_out/c5_fetch gpurun_out/c5_write "track_run_kernel<11, 3" gpurun_out/traffic_cfg5.json \
        "tools/track_only.py 1000 90000 11 32 (32 ch x 11 taps: one persistent launch = 9000 10-ms steps, virtual blocks). Below the algorithmic 2 B/channel-sample: the 32 channels read the same record region within ~1 ms of each other, so most IF lines are L2 / MALL hits" || exit 1
      pmc c5_sq1 "$SQ1" python3 "$R/tools/track_only.py" 1000 400 11 32 || exit 1
      pmc c5_sq3 "$SQ3" python3 "$R/tools/track_only.py" 1000 400 11 32 || exit 1
      python3 tools/pmc_sq.py gpurun_out/cfg5_sq.json gpurun_out/c5_sq1 gpurun_out/c5_sq3 -- "track_run_kernel<11, 3" || exit 1
      rm -f gpurun_out/c5_*/**/*kernel_trace.csv ;;
    acqbatch)  # config-2 fp64 correlation vs pairs per batch (BATCHES), pipelined default
      for b in ${BATCHES:-28 40 55 75 116}; do
        ACQ_BATCH=$b timeout -k 10 200 python3 tools/acq_only.py > gpurun_out/acqbatch_$b.txt 2>&1 \
          && echo "batch=$b corr_ms $(grep -o "'acq_corr_ms': [0-9.]*" gpurun_out/acqbatch_$b.txt | cut -d' ' -f2 | tr '\n' ' ') $(grep -E '^(fbin|snr)' gpurun_out/acqbatch_$b.txt | md5sum | cut -c1-8)" \
          || { tail -20 gpurun_out/acqbatch_$b.txt; exit 1; }
      done ;;
    acqprof1)  # rocprofv3 kernel stats of the config-2 acquisition with its two passes in order on one
      # stream (ACQ_PIPE=1): per-kernel durations free of the default pipeline's overlap (tools/acq_bound.py)
      ( cd /tmp && export TMPDIR=/tmp && ACQ_PIPE=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/acq_onestream" -o run -- python3 "$R/tools/acq_only.py" ) > gpurun_out/acq_onestream.log 2>&1 || { tail -20 gpurun_out/acq_onestream.log; exit 1; }
      python3 tools/prof_summary.py gpurun_out/acq_onestream > gpurun_out/acq_onestream_summary.txt && head -8 gpurun_out/acq_onestream_summary.txt
      rm -f gpurun_out/acq_onestream/**/*kernel_trace.csv ;;
    acqpipe)  # split correlator: batches on one stream vs pipelined over two (ACQ_PIPE), cfg2 / cfg4, fp64 / fp32
      for c in 2 4; do for f in "" 1; do for p in 1 2; do
        echo "-- cfg$c fp32=${f:-0} pipe=$p"
        ACQ_CFG=$c ACQ_FP32=$f ACQ_PIPE=$p timeout -k 10 200 python3 tools/acq_only.py > gpurun_out/acqpipe_${c}_${f:-0}_$p.txt 2>&1 \
          && grep -E "acq wall|^sv" gpurun_out/acqpipe_${c}_${f:-0}_$p.txt | tail -2 | cut -c1-400 || { tail -20 gpurun_out/acqpipe_${c}_${f:-0}_$p.txt; exit 1; }
      done; done; done ;;
    acqmask)  # config-2 fp64 correlation vs GNSS_OPT_ACQ_PIPE (1 one stream, 2 two streams; PIPES="1 2")
      for p in ${PIPES:-1 2 3 4 5 6}; do
        ACQ_PIPE=$p timeout -k 10 200 python3 tools/acq_only.py > gpurun_out/acqmask_$p.txt 2>&1 \
          && echo "pipe=$p corr_ms $(grep -o "'acq_corr_ms': [0-9.]*" gpurun_out/acqmask_$p.txt | cut -d' ' -f2 | tr '\n' ' ') fine_ms $(grep -o "'acq_fine_ms': [0-9.]*" gpurun_out/acqmask_$p.txt | cut -d' ' -f2 | tr '\n' ' ') $(grep -E '^(fbin|snr)' gpurun_out/acqmask_$p.txt | md5sum | cut -c1-8)" \
          || { tail -20 gpurun_out/acqmask_$p.txt; exit 1; }
      done ;;
    probes)  # timing-probe libraries (tools/build_probe.sh $PROBES): fp64 / VALU counts + stamps each
      for n in ${PROBES:-0}; do
        GNSS_LIB=$R/tools/probe_lib/libgnss_probe$n.so pmc pr${n}_sq "$SQ3" python3 "$R/tools/track_only.py" 1000 400 || exit 1
        python3 tools/pmc_sq.py gpurun_out/probe_sq_$n.json gpurun_out/pr${n}_sq -- "track_run_kernel<3, 3, false, false>" > /dev/null || exit 1
        GNSS_LIB=$R/tools/probe_lib/libgnss_probe$n.so GNSS_STAMPS=gpurun_out/st_$n.bin timeout -k 10 120 python3 tools/track_only.py 1000 2000 > gpurun_out/st_$n.log 2>&1 || { tail gpurun_out/st_$n.log; exit 1; }
        echo "probe $n: $(python3 tools/stamps_run.py gpurun_out/st_$n.bin | grep -E 'period|computed|all partials|next desc' | tr -s ' ' | tr '\n' ';')"
        rm -f gpurun_out/st_$n.bin  # (tens of MB: gpurun_out is copied back only below 64 MiB)
      done
      rm -f gpurun_out/pr*_sq/**/*kernel_trace.csv ;;
    probes1)
      for n in ${PROBES:-0}; do
        GNSS_LIB=$R/tools/probe_lib/libgnss_probe$n.so GNSS_STAMPS=gpurun_out/st1_$n.bin TRK_ITERS=1 timeout -k 10 120 python3 tools/track_only.py 1000 0 > gpurun_out/st1_$n.log 2>&1 || { tail gpurun_out/st1_$n.log; exit 1; }
        echo "== probe $n (1-ms phase)"; python3 tools/stamps_run.py gpurun_out/st1_$n.bin | grep -E "start ->|computed ->|partial out ->|all in ->|period \(|blk0 tail|lane:"
        rm -f gpurun_out/st1_$n.bin
      done ;;
    ab)  # A/B of library builds (tools/build_commit_lib.sh / build_probe.sh): AB="name ..." ->
         # tools/probe_lib/libgnss_<name>.so; 8-channel trackingCT (1000 ms + 4000 x 10 ms), per-launch
         # hipEvents and GNSS_STAMPS of the 10-ms launch (AB_TAPS=11 AB_NCH=32: the config-5 shape)
      for v in $AB; do
        GNSS_LIB=$R/tools/probe_lib/libgnss_$v.so TRK_HASH=1 TRK_PROFILE=1 TRK_ITERS=3 timeout -k 10 120 python3 tools/track_only.py 1000 40000 ${AB_TAPS:-3} ${AB_NCH:-8} > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
        echo "ab $v: $(grep -E 'track10|sha256' gpurun_out/ab_$v.log | tail -3 | tr '\n' ' ')"
        [ -n "$AB_NOSTAMPS" ] && continue
        GNSS_LIB=$R/tools/probe_lib/libgnss_$v.so GNSS_STAMPS=gpurun_out/abst_$v.bin TRK_ITERS=1 timeout -k 10 120 python3 tools/track_only.py 1000 2000 ${AB_TAPS:-3} ${AB_NCH:-8} > /dev/null 2>&1 || exit 1
        python3 tools/stamps_run.py gpurun_out/abst_$v.bin | grep -E "period|computed|all partials|next desc|tail" | sed "s/^/   /"
        rm -f gpurun_out/abst_$v.bin
      done ;;
    vt)  # vector tracking, 5 000 EKF-driven 1-ms steps of the reference's 5 channels (tools/vt_only.py)
      timeout -k 10 300 python3 tools/vt_only.py ${VT_ARGS} > gpurun_out/vt_only.txt 2>&1 && cat gpurun_out/vt_only.txt || { tail -20 gpurun_out/vt_only.txt; exit 1; } ;;
    geom)  # the 10-ms launch by channels x lane span: GEOM="nch:sub ..." (sub 0 = the engine's), 1000 ms + 4000 x 10 ms
      for g in ${GEOM:-1:0 1:2 1:1 8:0}; do
        n=${g%%:*}; u=${g##*:}
        TRK_SUB=$( [ "$u" != 0 ] && echo $u ) TRK_HASH=1 TRK_PROFILE=1 TRK_ITERS=2 timeout -k 10 120 python3 tools/track_only.py 1000 40000 3 $n > gpurun_out/geom_${n}_$u.log 2>&1 \
          && echo "geom nch=$n sub=$u: $(grep -E 'track10|sha256' gpurun_out/geom_${n}_$u.log | tail -2 | tr '\n' ' ')" || { tail -5 gpurun_out/geom_${n}_$u.log; exit 1; }
      done ;;
    c5geom)  # config-5 shape by channel count: 11 taps, 1000 ms + 9000 x 10 ms, C5NCH="1 4 8 32" channels
      for n in ${C5NCH:-1 4 8 32}; do
        TRK_HASH=1 TRK_PROFILE=1 TRK_ITERS=2 timeout -k 10 150 python3 tools/track_only.py 1000 90000 11 $n > gpurun_out/c5geom_$n.log 2>&1 \
          && echo "c5geom nch=$n: $(grep -E 'track10|sha256' gpurun_out/c5geom_$n.log | tail -2 | tr '\n' ' ')" || { tail -5 gpurun_out/c5geom_$n.log; exit 1; }
      done ;;
    xstamps)  # per-block stamps + SQ counters of probe-build variants (AB="pspread pxl"): tools/stamps_blocks.py
      for v in $AB; do
        L=$R/tools/probe_lib/libgnss_$v.so
        GNSS_LIB=$L GNSS_STAMPS=gpurun_out/xst_$v.bin TRK_ITERS=1 timeout -k 10 120 python3 tools/track_only.py 1000 2000 > gpurun_out/xst_$v.log 2>&1 || { tail -5 gpurun_out/xst_$v.log; exit 1; }
        echo "== $v"; python3 tools/stamps_run.py gpurun_out/xst_$v.bin | grep -E "period|computed|all partials|next desc|tail:" | sed "s/^/   /"
        python3 tools/stamps_blocks.py gpurun_out/xst_$v.bin 96 | sed "s/^/   /"
        rm -f gpurun_out/xst_$v.bin
        GNSS_LIB=$L pmc xsq1_$v "$SQ1" python3 "$R/tools/track_only.py" 1000 400 || exit 1
        GNSS_LIB=$L pmc xsq2_$v "$SQ2" python3 "$R/tools/track_only.py" 1000 400 || exit 1
        python3 tools/pmc_sq.py gpurun_out/xsq_$v.json gpurun_out/xsq1_$v gpurun_out/xsq2_$v -- "track_run_kernel<3, 3, false, false>" > /dev/null || exit 1
        python3 -c "import json; d=json.load(open('gpurun_out/xsq_$v.json')); k=[x for x in d if not x.startswith('_')][0]; print('   SQ', {c: round(w['median_per_dispatch']) for c, w in d[k].items() if isinstance(w, dict) and 'median_per_dispatch' in w})" | cut -c1-1200
        rm -f gpurun_out/xsq*_$v/**/*kernel_trace.csv
      done ;;
    acqpair)  # config-2 fp64 correlation by ACQ_PIPE:front (GNSS_PAIR_FRONT, probe library PAIRLIB):
              # PAIRS="2:60 3:100 3:60 3:40" -> corr_ms of the three calls and a digest of the decisions
      for v in ${PAIRS:-2:60 3:100 3:60 3:40}; do
        pp=${v%%:*}; fr=${v##*:}
        GNSS_LIB=$R/tools/probe_lib/libgnss_${PAIRLIB:-pair}.so ACQ_PIPE=$pp GNSS_PAIR_FRONT=$fr timeout -k 10 200 python3 tools/acq_only.py > gpurun_out/acqpair_${pp}_$fr.txt 2>&1 \
          && echo "acqpair pipe=$pp front=$fr: corr_ms $(grep -o "'acq_corr_ms': [0-9.]*" gpurun_out/acqpair_${pp}_$fr.txt | cut -d' ' -f2 | tr '\n' ' ') acq_ms $(grep -o "'acq_ms': [0-9.]*" gpurun_out/acqpair_${pp}_$fr.txt | cut -d' ' -f2 | tr '\n' ' ') $(grep -E '^(fbin|snr|sv)' gpurun_out/acqpair_${pp}_$fr.txt | md5sum | cut -c1-8)" \
          || { tail -5 gpurun_out/acqpair_${pp}_$fr.txt; exit 1; }
      done ;;
    acqlib)  # config-2 acquisition (tools/acq_only.py, fp64) under each library of ACQLIBS (tools/probe_lib/libgnss_<name>.so,
             # "prod" = the product): correlation ms of the three calls and a digest of the decisions
      for v in ${ACQLIBS:-prod}; do
        L=$R/assignment-for-aae6102_gnss-sdr_amd/lib/libgnss_mi355x.so; [ "$v" != prod ] && L=$R/tools/probe_lib/libgnss_$v.so
        GNSS_LIB=$L timeout -k 10 200 python3 tools/acq_only.py > gpurun_out/acqlib_$v.txt 2>&1 \
          && echo "acqlib $v: corr_ms $(grep -o "'acq_corr_ms': [0-9.]*" gpurun_out/acqlib_$v.txt | cut -d' ' -f2 | tr '\n' ' ') acq_ms $(grep -o "'acq_ms': [0-9.]*" gpurun_out/acqlib_$v.txt | cut -d' ' -f2 | tr '\n' ' ') $(grep -E '^(fbin|snr|sv)' gpurun_out/acqlib_$v.txt | md5sum | cut -c1-8)" \
          || { tail -20 gpurun_out/acqlib_$v.txt; exit 1; }
      done ;;
    vtab)  # tools/vt_only.py under each library of VTLIBS (tools/probe_lib/libgnss_<name>.so; "prod" = the
           # product) and each VT_NB of VTNBS (blocks per channel)
      for v in ${VTLIBS:-prod}; do for nb in ${VTNBS:-0}; do
        L=$R/assignment-for-aae6102_gnss-sdr_amd/lib/libgnss_mi355x.so; [ "$v" != prod ] && L=$R/tools/probe_lib/libgnss_$v.so
        GNSS_LIB=$L VT_NB=$( [ "$nb" != 0 ] && echo $nb ) timeout -k 10 120 python3 tools/vt_only.py 2000 2 > gpurun_out/vtab_${v}_$nb.txt 2>&1 \
          && echo "vtab $v nb=$nb: $(grep '^vt ' gpurun_out/vtab_${v}_$nb.txt | tail -1 | cut -c1-110)" || { tail -5 gpurun_out/vtab_${v}_$nb.txt; exit 1; }
      done; done ;;
    vtprof)  # rocprofv3 kernel stats of tools/vt_only.py (1 000 steps, one iteration)
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/vtprof" -o run -- python3 "$R/tools/vt_only.py" 1000 1 ) > gpurun_out/vtprof.log 2>&1 || { tail -20 gpurun_out/vtprof.log; exit 1; }
      python3 tools/prof_summary.py gpurun_out/vtprof > gpurun_out/vtprof_summary.txt && head -8 gpurun_out/vtprof_summary.txt
      rm -f gpurun_out/vtprof/**/*kernel_trace.csv ;;
    lat)  # fp64 / fp32 dependent-latency micro-benchmark (tools/micro/lat2, built in-tree)
      timeout -k 10 60 ./tools/micro/lat2 > gpurun_out/lat2.txt 2>&1 && cat gpurun_out/lat2.txt || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
