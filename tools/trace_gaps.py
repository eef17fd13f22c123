"""Timeline of one stream from a rocprofv3 kernel (+ memory copy) trace (development tool).

  python tools/trace_gaps.py <trace dir> [kernel-name filter] [last N entries]

Prints each kernel / copy with its duration and the idle gap before it, then a summary of busy
vs idle time over the window (the BA driver's LM iterations: how much of an iteration is kernel
time and how much is launch gaps and host round trips).
"""
import csv
import gzip
import re
import sys
from pathlib import Path


def rows(path):
    op = gzip.open if str(path).endswith(".gz") else open
    with op(path, "rt") as f:
        yield from csv.DictReader(f)


def short(name):
    m = re.search(r"::([A-Za-z0-9_]+)(?:<[^(]*>)?\(", name)
    return m.group(1) if m else name.split("(")[0][:40]


def main():
    d = Path(sys.argv[1])
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    last = int(sys.argv[3]) if len(sys.argv) > 3 else 120
    ev = []
    for p in list(d.rglob("*kernel_trace.csv*")):
        for r in rows(p):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    for p in list(d.rglob("*memory_copy_trace.csv*")):
        for r in rows(p):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy:" + r.get("Direction", "?")))
    ev.sort()
    if filt:
        ev = [e for e in ev if filt in e[2] or e[2].startswith("copy")]
    ev = ev[-last:]
    busy = idle = 0
    prev = None
    for s, e, n in ev:
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        print(f"{n:28s} {((e - s) / 1e3):8.1f} us   gap {gap:7.1f} us")
        if prev is not None:
            idle += max(0, s - prev)
        busy += e - s
        prev = max(prev or 0, e)
    print(f"window {len(ev)} entries: busy {busy / 1e3:.1f} us, idle {idle / 1e3:.1f} us")


if __name__ == "__main__":
    main()
