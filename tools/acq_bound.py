"""What bounds the fp64 acquisition kernels, from this round's PMC passes
(profiles/r02_acq_counters.json: FETCH_SIZE / WRITE_SIZE / SQ counters, median per
dispatch) and the rocprofv3 kernel-trace averages of the bench
(profiles/r02_bench_kernel_summary.txt). HBM bytes = FETCH_SIZE x 2 + WRITE_SIZE (KB;
MI355X_MICROARCH.md HBM section). Writes profiles/acq_bound_r02.json (read by bench.py)."""
import json, os, re, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cnt = json.load(open(os.path.join(ROOT, "profiles", "r02_acq_counters.json")))
summ = open(os.path.join(ROOT, "profiles", "r02_bench_kernel_summary.txt")).read().splitlines()


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
    ck = next(k for k in cnt if k.startswith(key.split("<")[0]) and (("f64" in k) == ("f64" in key)))
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
    e["bound"] = ("hbm (streaming writes of the batch intermediate)" if e["hbm_frac"] and e["hbm_frac"] > 0.4
                  else "lds issue (fp64 2000-point Stockham passes in LDS)" if e["wait_inst_lds_frac"] > 0.2
                  else "latency (waves parked on loads / barriers)")
    out[key] = e
json.dump(out, open(os.path.join(ROOT, "profiles", "acq_bound_r02.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
