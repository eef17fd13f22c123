"""Per-variant SQ counter table of a tools/abl.py run under rocprofv3 --pmc (development tool).

  python tools/abl_pmc_table.py gpurun_out/abl_pmc/run_counter_collection.csv v1,v2,... [kernel]

abl.py runs 13 steps per variant (3 warm-up + 10 timed); the first 3 launches of each variant are
skipped.  Prints per-wave instruction counts of the kernel (default fast_nms).
"""
import collections
import csv
import sys

path, names = sys.argv[1], sys.argv[2].split(",")
kern = sys.argv[3] if len(sys.argv) > 3 else "fast_nms"
rows = [r for r in csv.DictReader(open(path)) if kern in r["Kernel_Name"]]
d = collections.OrderedDict()
for r in rows:
    e = d.setdefault(int(r["Dispatch_Id"]), {"vgpr": r["VGPR_Count"], "lds": r["LDS_Block_Size"]})
    e[r["Counter_Name"]] = float(r["Counter_Value"])
ids = sorted(d)
per = len(ids) // len(names)
for i, n in enumerate(names):
    ch = [d[k] for k in ids[i * per:(i + 1) * per]][3:]
    keys = [c for c in ch[0] if c.startswith("SQ_")]
    avg = {c: sum(x[c] for x in ch) / len(ch) for c in keys}
    w = avg.get("SQ_WAVES", 1.0)
    print(f"{n:10s} vgpr {ch[0]['vgpr']:>3} lds {ch[0]['lds']:>6} " +
          " ".join(f"{c[3:]}/w {avg[c] / w:.0f}" for c in keys if c != "SQ_WAVES") + f" waves {w:.0f}")
