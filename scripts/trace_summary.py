"""Summarise a rocprofv3 ``--kernel-trace`` run: per (kernel, grid) the dispatch count and the
average / minimum duration, with the code object's LDS, VGPR and scratch sizes.
``python scripts/trace_summary.py gpurun_out/prof [out.txt]``."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d, out=None):
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = defaultdict(list)
    meta = {}
    for fn in files:
        for r in csv.DictReader(open(fn)):
            lds = r.get("LDS_Block_Size", r.get("Lds_Size", "?"))
            key = (r["Kernel_Name"], int(r["Grid_Size_X"] if "Grid_Size_X" in r else r.get("Grid_Size", 0)), lds)
            rows[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
            meta[key] = (r.get("LDS_Block_Size", r.get("Lds_Size", "?")), r.get("VGPR_Count", r.get("Arch_VGPR_Count", "?")),
                         r.get("Scratch_Size", r.get("Private_Segment_Size", "?")))
    lines = []
    for key, ms in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        lds, vgpr, scr = meta[key]
        lines.append(f"{key[0][:40]:40s} grid {key[1]:8d} LDS {lds:>6} VGPR {vgpr:>4} scratch {scr:>5}: "
                     f"{len(ms)} dispatches, avg {sum(ms) / len(ms):.3f} ms, min {min(ms):.3f} ms")
    text = "\n".join(lines)
    print(text)
    if out:
        with open(out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
