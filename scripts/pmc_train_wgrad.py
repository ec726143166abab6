"""Summarise scripts/pmc_train_wgrad.sh: HBM bytes and counters per launch of the training step's
dominant launch (wgrad_tr_kernel + reduce_partials_kernel of cista_wgrad_ista_p).  gfx950 read
correction as scripts/pmc_traffic.py (read = 2 x FETCH_SIZE KiB, WRITE_SIZE exact).
usage: python scripts/pmc_train_wgrad.py out.json"""
import collections
import csv
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"wgrad_tr_kernel": "wgrad_tr_kernel", "reduce_partials_kernel": "reduce_partials_kernel"}


def main(out):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", "pmctw_*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = next((v for n, v in KERNELS.items() if n in r["Kernel_Name"]), None)
            if k is None:
                continue
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    per = {}
    total = 0
    for k, d in vals.items():
        m = {c: sum(v) / len(v) for c, v in d.items()}
        e = {"mean_dur_us_profiled": round(sum(durs[k]) / len(durs[k]), 2),
             "counters": {c: round(v, 1) for c, v in m.items()}}
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            e["hbm_bytes_per_launch"] = round((2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024)
            total += e["hbm_bytes_per_launch"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
            # busy cycles summed over 1024 SIMDs vs the per-XCD active cycles summed over 8 XCDs
            e["mfma_busy_frac"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (m["GRBM_GUI_ACTIVE"] / 8), 4)
        if "SQ_LDS_BANK_CONFLICT" in m and "SQ_ACTIVE_INST_LDS" in m and m["SQ_ACTIVE_INST_LDS"] > 0:
            e["lds_conflict_per_active_inst"] = round(m["SQ_LDS_BANK_CONFLICT"] / m["SQ_ACTIVE_INST_LDS"], 4)
        per[k] = e
    lib = os.path.join(ROOT, "v2e2v_amd", "libcista_hip.so")
    res = {"source": "scripts/pmc_train_wgrad.sh (rocprofv3 --pmc, one counter group per pass)",
           "correction": "read = 2 x FETCH_SIZE (gfx950), KiB -> bytes",
           "lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(),
           "kernels": per,
           "layers": {"ista_P_wgrad": {"hbm_bytes_per_launch": total}}}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
