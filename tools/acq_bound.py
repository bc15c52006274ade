"""What bounds the fp64 acquisition kernels, from a round's PMC passes
(profiles/rNN_acq_counters.json: FETCH_SIZE / WRITE_SIZE / SQ counters, median per
dispatch; tools/gpu.sh acqpmc) and the rocprofv3 kernel-trace averages of the bench
(profiles/rNN_bench_kernel_summary.txt; tools/gpu.sh prof). HBM bytes = FETCH_SIZE x 2 +
WRITE_SIZE (KB; MI355X_MICROARCH.md HBM section). Writes profiles/acq_bound_rNN.json (read
by bench.py), stamped with the source digest the counters were taken at.
Usage: python3 tools/acq_bound.py [NN]   (default 03)"""
import json, os, re, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RN = sys.argv[1] if len(sys.argv) > 1 else "03"
cnt = json.load(open(os.path.join(ROOT, "profiles", f"r{RN}_acq_counters.json")))
# per-kernel durations: the one-stream order's kernel stats when present (tools/gpu.sh acqprof1;
# the default pipelines batch b's row pass beside b+1's column pass, so the bench's kernel-trace
# durations overlap and would understate each kernel's rate), else the bench's summary
_one = os.path.join(ROOT, "profiles", f"r{RN}_acq_onestream_kernel_summary.txt")
DUR_SRC = _one if os.path.exists(_one) else os.path.join(ROOT, "profiles", f"r{RN}_bench_kernel_summary.txt")
summ = open(DUR_SRC).read().splitlines()
meta = cnt.pop("_meta", {})


def avg_us(sub):
    for ln in summ:
        if sub in ln:
            return float(re.split(r"\s+", ln.strip())[-3])
    return None


out = {}
for key, sub in (("inv_cols_kernel<29, double2>", "inv_cols_kernel<29, HIP_vector_type<"),
                 ("inv_rows_kernel_f64<29>", "inv_rows_kernel_f64<29>"),
                 ("fine_rows_kernel<29>", "fine_rows_kernel<29"),
                 ("fine_cols_kernel<29>", "fine_cols_kernel<29>")):
    ck = next((k for k in cnt if k.startswith(key.split("<")[0]) and (("f64" in k) == ("f64" in key))
               and cnt[k]), None)
    if ck is None:
        continue
    c = {n: v["median_per_dispatch"] for n, v in cnt[ck].items()}
    us = avg_us(sub)
    hbm = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
    wave = c["SQ_WAVE_CYCLES"]
    lds = c["SQ_LDS_IDX_ACTIVE"]
    e = {"avg_launch_us": us, "hbm_bytes_per_launch": hbm,
         "hbm_GBs": round(hbm / (us * 1e-6) / 1e9, 1) if us else None,
         "hbm_frac": round(hbm / (us * 1e-6) / 8e12, 3) if us else None,
         "wait_any_frac": round(c["SQ_WAIT_ANY"] / wave, 3),
         "wait_inst_lds_frac": round(c["SQ_WAIT_INST_LDS"] / wave, 3),
         "valu_active_frac": round(c["SQ_ACTIVE_INST_VALU"] / wave, 3),
         "lds_bank_conflict_frac": round(c["SQ_LDS_BANK_CONFLICT"] / lds, 3) if lds else 0.0}
    writes = c.get("WRITE_SIZE", 0.0) * 1024.0 > 0.5 * hbm  # (mostly a write stream)
    e["bound"] = ("hbm (streaming writes of the batch intermediate)" if e["hbm_frac"] and e["hbm_frac"] > 0.5 and writes
                  else "hbm read + fp64 Stockham passes in LDS" if e["hbm_frac"] and e["hbm_frac"] > 0.4
                  and e["wait_inst_lds_frac"] > 0.1
                  else "lds issue (fp64 2000-point Stockham passes in LDS)" if e["wait_inst_lds_frac"] > 0.2
                  else "latency (waves parked on loads / barriers)")
    out[key] = e
# the correlator's bytes per call against the models (config 2: 1.0764e9 hypothesis-samples
# per call, 17 batches): SURVEY 8d's 16 B per hypothesis-sample (an fp32 product spectrum
# read + an fp32 accumulator read and write) and its fp64 restatement, 32 B (the
# reference's precision: a complex-fp64 spectrum read + an fp64 accumulator read and write)
if "inv_cols_kernel<29, double2>" in out and "inv_rows_kernel_f64<29>" in out:
    units, nbat = 1.0764e9, 17
    per_call = nbat * (out["inv_cols_kernel<29, double2>"]["hbm_bytes_per_launch"]
                       + out["inv_rows_kernel_f64<29>"]["hbm_bytes_per_launch"])
    out["correlator_per_call"] = {"hbm_bytes": per_call, "batches": nbat,
                                  "model_fp32_16B": 16 * units, "x_model_fp32": round(per_call / (16 * units), 3),
                                  "model_fp64_32B": 32 * units, "x_model_fp64": round(per_call / (32 * units), 3)}
meta["durations_from"] = os.path.relpath(DUR_SRC, ROOT)
out["_meta"] = meta
json.dump(out, open(os.path.join(ROOT, "profiles", f"acq_bound_r{RN}.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
