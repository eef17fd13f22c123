"""Per-variant averages of the fast_nms counters from tools/abl_pmc.sh (dev tool).
usage: python tools/abl_pmc_table.py <variants csv>"""
import collections
import csv
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from rocprof_summary import short  # noqa: E402

V = sys.argv[1].split(",")
rows = [r for r in csv.DictReader(open("gpurun_out/abl_pmc/run_counter_collection.csv"))
        if short(r["Kernel_Name"]) == "fast_nms_kernel"]
byd = collections.defaultdict(dict)
for r in rows:
    byd[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
ds = sorted(byd)
for vi, v in enumerate(V):
    sel = ds[vi * 13 + 3:(vi + 1) * 13]
    avg = {k: sum(byd[d][k] for d in sel) / len(sel) for k in byd[sel[0]]}
    w = avg["SQ_WAVES"]
    print(f"{v:>5}", {k.replace("SQ_", ""): round(x / w) for k, x in sorted(avg.items()) if k != "SQ_WAVES"})
