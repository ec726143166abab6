"""Per-stream activity of a rocprofv3 --kernel-trace CSV (the training backward's side-stream
weight gradients): for each stream, busy time (union of its kernels' intervals), and the time
during which both streams had a kernel running; plus the gaps on the main stream.
usage: python scripts/stream_timeline.py TRACE.csv"""
import csv
import sys
from collections import defaultdict


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def inter(x, y):
    i = j = 0
    tot = 0
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        tot += max(0, b - a)
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    by = defaultdict(list)
    names = defaultdict(lambda: defaultdict(float))
    for r in rows:
        key = (r["Queue_Id"], r["Stream_Id"])
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        by[key].append((a, b))
        names[key][r["Kernel_Name"].split("(")[0][:60]] += (b - a) / 1e6
    t0 = min(a for v in by.values() for a, _ in v)
    t1 = max(b for v in by.values() for _, b in v)
    print(f"span {(t1 - t0) / 1e6:.2f} ms")
    u = {k: union(v) for k, v in by.items()}
    for k, v in sorted(u.items(), key=lambda kv: -sum(b - a for a, b in kv[1])):
        busy = sum(b - a for a, b in v)
        top = sorted(names[k].items(), key=lambda x: -x[1])[:4]
        print(f"queue {k[0]} stream {k[1]}: {len(by[k])} kernels, busy {busy / 1e6:.2f} ms; top "
              + ", ".join(f"{n} {t:.2f}" for n, t in top))
    ks = sorted(u, key=lambda k: -sum(b - a for a, b in u[k]))
    if len(ks) >= 2:
        print(f"overlap of the two busiest streams: {inter(u[ks[0]], u[ks[1]]) / 1e6:.2f} ms")
        allu = union([iv for k in ks for iv in (tuple(x) for x in u[k])])
        print(f"any stream busy: {sum(b - a for a, b in allu) / 1e6:.2f} ms of {(t1 - t0) / 1e6:.2f}")


if __name__ == "__main__":
    main()
