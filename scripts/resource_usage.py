"""Per-kernel register / scratch report from a hipcc -Rpass-analysis=kernel-resource-usage log.

usage: python scripts/resource_usage.py LOG [--all]   (lists kernels with scratch unless --all)
"""
import re
import sys


def parse(path):
    txt = open(path).read()
    rows = []
    for b in re.split(r'remark: .*?Function Name: ', txt)[1:]:
        name = b.split('\n')[0].split(' [-Rpass')[0].strip()

        def g(k):
            m = re.search(k + r': (\d+)', b)
            return int(m.group(1)) if m else -1
        rows.append((name, g('VGPRs'), g(r'ScratchSize \[bytes/lane\]'), g('VGPRs Spill'),
                     g(r'Occupancy \[waves/SIMD\]')))
    return rows


if __name__ == "__main__":
    rows = parse(sys.argv[1])
    show_all = "--all" in sys.argv
    print(f"{len(rows)} kernels, {sum(r[2] > 0 for r in rows)} with scratch")
    for r in rows:
        if show_all or r[2] > 0:
            print(f"vgpr {r[1]:4d} scratch {r[2]:4d} spill {r[3]:3d} occ {r[4]}  {r[0]}")
