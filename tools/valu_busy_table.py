"""VALU issue-occupancy calibration table (development tool; run here on gpurun_out/ of tools/gr_vbusy.sh).

  python tools/valu_busy_table.py gpurun_out/vbusy > profiles/r5_valu_probe_pmc.md

For every probe<OP> launch of tools/valu_probe.hip (one wave-instruction form, 8 independent chains,
1/2/4 waves per SIMD) and for every kernel of the headline ORB leg it prints
  dual/I  = SQ_ACTIVE_INST_VALU2 / SQ_INSTS_VALU (share of instructions issued as the second of a
            dual-issue quad-cycle: one instruction from each of two waves, both full-rate forms)
  busy    = (SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2) x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
  I/cyc   = SQ_INSTS_VALU per SIMD per cycle
so the busy metric of tools/rocprof_summary.py is checked against loops whose issue is known.
"""
import csv
import re
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from rocprof_summary import N_SIMD, N_XCD, valu_busy  # noqa: E402


def load(d: Path):
    rows, name = defaultdict(dict), {}
    for r in csv.DictReader(open(d / "run_counter_collection.csv")):
        i = int(r["Dispatch_Id"])
        rows[i][r["Counter_Name"]] = float(r["Counter_Value"])
        name[i] = r["Kernel_Name"]
    dur = {int(r["Dispatch_Id"]): int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
           for r in csv.DictReader(open(d / "run_kernel_trace.csv"))}
    return rows, name, dur


def kname(n):
    n = n.replace("(anonymous namespace)::", "")
    return re.match(r"(?:void )?([\w:]+)", n).group(1).split("::")[-1]


def main():
    root = Path(sys.argv[1])
    rows, name, dur = load(root / "probe")
    ops = [l.split()[0] for l in open(root / "probe.txt") if " w1:" in l]
    disp = [i for i in sorted(rows) if "probe" in name[i]]
    print("# VALU issue occupancy — calibration on tools/valu_probe.hip (round 5)\n")
    print("One `rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU SQ_BUSY_CU_CYCLES "
          "SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace` pass (tools/gr_vbusy.sh).  Each probe launch runs one "
          "instruction form (8 independent chains x 16 unrolled, 2000 iterations) on 256 workgroups "
          "(one per CU); second launch of each (waves per SIMD) pair shown.  SQ_ACTIVE_INST_VALU / "
          "SQ_INSTS_VALU is 1.000 for every form (it counts issues, not busy cycles).\n")
    print("| form | waves/SIMD | µs | clock GHz (GRBM/8/µs) | dual/I | I per SIMD-cycle | busy |")
    print("|---|---|---|---|---|---|---|")
    for j, i in enumerate(disp):
        if j % 2 == 0:
            continue
        c, t = rows[i], dur[i]
        w = (1, 2, 4)[(j // 2) % 3]
        I, V2, G = c["SQ_INSTS_VALU"], c["SQ_ACTIVE_INST_VALU2"], c["GRBM_GUI_ACTIVE"]
        print(f"| {ops[j // 6]} | {w} | {t / 1e3:.1f} | {G / N_XCD / t:.2f} | {V2 / I:.3f} | "
              f"{I / N_SIMD / (G / N_XCD):.3f} | {valu_busy(I, V2, G):.3f} |")
    print("\nFull-rate forms (VOP2 f32/u32/b32/u16/f16 add, mul, fma, logic, lshr, mov, bitop3) dual-issue "
          "from two waves (~0.42 per SIMD-cycle at 2+ waves); VOP3-only and packed forms do not (~0.24). "
          "Both saturate `busy` at 0.93-0.95.\n")
    rows, name, dur = load(root / "orb")
    agg = defaultdict(list)
    for i in sorted(rows):
        if i in dur and "GRBM_GUI_ACTIVE" in rows[i] and "SQ_INSTS_VALU" in rows[i]:
            agg[kname(name[i])].append((rows[i], dur[i]))
    print("## Headline ORB leg (`bench.py --no-ba --no-pose --no-tracking`, first 3 launches per kernel skipped)\n")
    print("| kernel | launches | avg µs | dual/I | busy |")
    print("|---|---|---|---|---|")
    for k, l in agg.items():
        l = l[3:] if len(l) > 6 else l
        I = sum(c["SQ_INSTS_VALU"] for c, _ in l)
        V2 = sum(c["SQ_ACTIVE_INST_VALU2"] for c, _ in l)
        G = sum(c["GRBM_GUI_ACTIVE"] for c, _ in l)
        T = sum(t for _, t in l)
        if I == 0 or T / len(l) < 20e3:
            continue
        print(f"| {k} | {len(l)} | {T / len(l) / 1e3:.1f} | {V2 / I:.3f} | {valu_busy(I, V2, G):.3f} |")


if __name__ == "__main__":
    main()
