"""Average counters per kernel from rocprofv3 --pmc run_counter_collection.csv files (dev tool).
usage: python tools/pmc_table.py <dir> [<dir> ...]"""
import collections
import csv
import gzip
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from rocprof_summary import short  # noqa: E402

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    p = Path(d) / "run_counter_collection.csv"
    f = gzip.open(str(p) + ".gz", "rt") if not p.exists() else open(p)
    for r in csv.DictReader(f):
        agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in sorted(agg.items()):
    if k.startswith("__amd") or "Ops" in k or "copy" in k:
        continue
    print(k, "n=%d" % len(next(iter(c.values()))))
    for n, v in sorted(c.items()):
        print(f"   {n:24s} {sum(v) / len(v):16.0f}")
