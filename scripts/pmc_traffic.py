"""HBM traffic per kernel launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE reports exactly half the bytes of a
wide (16 B/lane) coalesced read, which is what every staging / epilogue read of these kernels
is, so read bytes = 2 * FETCH_SIZE; WRITE_SIZE is exact for 16 B/lane stores.  Both counters
are in KiB and were collected in separate passes (they cannot share the 4 TCC slots).

A layer may run as several dispatches of one kernel (the two-region tiling of plan_tiles: an
exact-width region and a column strip, different grid sizes): the counters and durations are
averaged per (layer, grid size) and summed over the grid sizes, i.e. reported per layer
launch (what bench.py times with HIP events).

usage: python scripts/pmc_traffic.py 'gpurun_out/pmcl_*/run_counter_collection.csv' out.json [lib.so]
The library's sha256 is recorded: bench.py only quotes the traffic for the build it measured.
"""
import hashlib
import os
import collections
import csv
import glob
import json
import re
import sys

# (STAGE, EPI) template arguments of conv3x3_split3 -> frame-schedule layer
CONV_LAYER = {(1, 0): "W0", (0, 0): "P0", (0, 4): "gates", (0, 5): "out_gates", (0, 2): "ista_D",
              (0, 3): "ista_P", (0, 1): "Dg", (0, 6): "lstm", (4, 9): "upsample", (2, 7): "upsample:border",
              (2, 1): "upsample", (5, 0): "input+W0:conv"}


def layer_of(name):
    m = re.search(r"conv3x3_split3<([^>]*)>", name)
    if m:
        args = [x.strip() for x in m.group(1).split(",")]
        kn = "conv3x3_split3<" + ",".join(args) + ">"
        if (int(args[4]), int(args[5])) == (0, 0) and args[:4] == ["6", "2", "2", "2"]:
            return "input+W0:conv", kn            # the 64-column bias conv over the s2d input
        return CONV_LAYER.get((int(args[4]), int(args[5]))), kn
    if "input_stage_kernel" in name:
        return "input", name.split("(")[0].replace("void ", "")
    if "s2d_input_kernel" in name:
        return "input+W0:s2d", name.split("(")[0].replace("void ", "")
    if "input_w0_kernel" in name or "input_border_kernel" in name:
        return "input+W0:border", name.split("(")[0].replace("void ", "")
    if "final_q_kernel" in name or "final_stage_kernel" in name:
        return "final", name.split("(")[0]
    return None, None


def lib_sha256(path):
    return hashlib.sha256(open(path, "rb").read()).hexdigest()


def main(pattern, out, lib=None):
    # (layer, grid size) -> counter -> values; (layer, grid size) -> durations (us)
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    names = {}
    for f in sorted(glob.glob(pattern)):
        for r in csv.DictReader(open(f)):
            layer, kname = layer_of(r["Kernel_Name"])
            if layer is None:
                continue
            names[layer] = kname
            key = (layer, int(r.get("Grid_Size", 0) or 0))
            vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            durs[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    mean = lambda v: sum(v) / len(v)
    res = {}
    for layer in sorted({k[0] for k in vals}):
        keys = sorted(k for k in vals if k[0] == layer)
        if any("FETCH_SIZE" not in vals[k] or "WRITE_SIZE" not in vals[k] for k in keys):
            continue
        fk = sum(mean(vals[k]["FETCH_SIZE"]) for k in keys)
        wk = sum(mean(vals[k]["WRITE_SIZE"]) for k in keys)
        res[layer] = {"kernel": names[layer], "dispatches": sum(len(vals[k]["FETCH_SIZE"]) for k in keys),
                      "grids_per_launch": [k[1] for k in keys],
                      "mean_dur_us_profiled": round(sum(mean(durs[k]) for k in keys), 2),
                      "FETCH_SIZE_KiB": round(fk, 1), "WRITE_SIZE_KiB": round(wk, 1),
                      "hbm_bytes_per_launch": round((2 * fk + wk) * 1024)}
    lib = lib or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "v2e2v_amd",
                              "libcista_hip.so")
    json.dump({"source": pattern, "correction": "read = 2 x FETCH_SIZE (gfx950), KiB -> bytes",
               "lib_sha256": lib_sha256(lib), "layers": res}, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
