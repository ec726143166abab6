"""Per-launch summary of a rocprofv3 --kernel-trace CSV: kernels grouped by (name, grid size),
with call counts, mean / min / max duration and share of the total.
usage: python scripts/trace_summary.py 'gpurun_out/trace_train/*kernel_trace.csv' [top]"""
import collections
import csv
import glob
import re
import sys


def short(name):
    m = re.search(r"conv3x3_split3<([^>]*)>", name)
    if m:
        return "conv<" + ",".join(x.strip() for x in m.group(1).split(",")) + ">"
    return name.split("(")[0].replace("void ", "").replace("cista::", "")


def main(pattern, top=40):
    d = collections.defaultdict(list)
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            key = (short(r["Kernel_Name"]), int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0))
            d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot = sum(sum(v) for v in d.values())
    rows = sorted(d.items(), key=lambda kv: -sum(kv[1]))
    print(f"total {tot / 1e3:.2f} ms over {sum(len(v) for v in d.values())} launches")
    for (name, grid), v in rows[:top]:
        print(f"{100 * sum(v) / tot:6.2f}% n={len(v):4d} mean {sum(v) / len(v):8.1f} us  min {min(v):8.1f}  max {max(v):8.1f}"
              f"  grid {grid:9d}  {name}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
