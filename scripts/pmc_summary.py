"""Summarise rocprofv3 --pmc CSVs (gpurun_out/pmcl_*/run_counter_collection.csv) per kernel:
per-dispatch mean of every counter, plus the kernel's mean duration from the kernel trace."""
import collections
import csv
import glob
import json
import re
import sys


def short(name):
    m = re.search(r"conv3x3_split3<([^>]*)>", name)
    if m:
        return "conv<" + m.group(1).replace(" ", "") + ">"
    m = re.search(r"cista::(\w+)", name)
    return "cista::" + m.group(1) if m else name[:40]


def main(pattern):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(pattern)):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {}
    for k, d in per.items():
        if "cista" not in k and "conv<" not in k:
            continue
        out[k] = {c: sum(v) / len(v) for c, v in d.items()}
        out[k]["dur_us"] = sum(dur[k]) / len(dur[k])
    return out


if __name__ == "__main__":
    res = main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcl_*/run_counter_collection.csv")
    print(json.dumps(res, indent=1))
