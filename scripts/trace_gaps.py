"""Summarise the idle time of a rocprofv3 ``--kernel-trace`` run: over a window of the run (the
dispatches from the first of ``START`` to the end), the GPU's busy time (union of kernel
intervals), the idle gaps between them by size, and the kernel count -- whether a launch-heavy
loop (a coordinated ADMM round's straggler iterations) is bound by the host's launch rate.
``python scripts/trace_gaps.py gpurun_out/prof [START_KERNEL_SUBSTRING]``."""
import csv
import glob
import os
import sys


def main(d, start=None):
    rows = []
    for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    if start:
        i0 = next((i for i, r in enumerate(rows) if start in r[2]), 0)
        rows = rows[i0:]
    if not rows:
        print("no dispatches")
        return
    busy, gaps, end = 0, [], rows[0][0]
    for s, e, _ in rows:
        if s > end:
            gaps.append(s - end)
        busy += max(0, e - max(s, end))
        end = max(end, e)
    span = end - rows[0][0]
    print(f"dispatches {len(rows)}, span {span / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms "
          f"({100 * busy / max(span, 1):.1f} %), idle {(span - busy) / 1e6:.3f} ms in {len(gaps)} gaps")
    for lo, hi in ((0, 2e3), (2e3, 10e3), (10e3, 50e3), (50e3, 1e12)):
        g = [x for x in gaps if lo <= x < hi]
        print(f"  gaps {lo / 1e3:6.0f}-{hi / 1e3:6.0f} us: {len(g):6d}, total {sum(g) / 1e6:8.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
