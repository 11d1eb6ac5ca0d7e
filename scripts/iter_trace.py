"""Per-iteration view of a coordinated ADMM round from a rocprofv3 ``--kernel-trace`` run: the
iterations are cut at ``mpcx_admm_block_stop`` (kernel k_block_stop) (one per iteration, after the residual totals);
for each iteration of the last ``ROUNDS`` rounds: wall span (from the previous stop's end), GPU busy
time (union of kernel intervals), the solve launches' durations, and the kernel count -- is a
straggler iteration bound by its solves or by the launches around them?
``python scripts/iter_trace.py gpurun_out/prof [rounds]``."""
import csv
import glob
import os
import sys


def main(d, rounds=1):
    rows = []
    for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)))
    rows.sort()
    stops = [i for i, r in enumerate(rows) if "k_block_stop" in r[2]]
    # a round starts with the stop of iteration 0 (the clock stamp): the stops whose previous kernel
    # is not a block_expand of the previous iteration are hard to tell apart, so rounds are cut at
    # gaps > 5 ms between consecutive stops (the untimed plant step between control steps)
    cuts = [0] + [k for k in range(1, len(stops)) if rows[stops[k]][0] - rows[stops[k - 1]][1] > 5e6] + [len(stops)]
    rnds = [stops[cuts[j]:cuts[j + 1]] for j in range(len(cuts) - 1)]
    for rs in rnds[-rounds:]:
        print(f"round of {len(rs) - 1} iterations")
        tot = {"span": 0, "busy": 0, "solve": 0, "n": 0}
        for a, b in zip(rs, rs[1:]):
            seg = rows[a + 1:b + 1]
            t0, t1 = rows[a][1], rows[b][1]
            busy, end = 0, t0
            for s, e, _, _ in seg:
                s = max(s, end)
                if e > s:
                    busy += e - s
                    end = e
            solves = [(e - s) / 1e3 for s, e, n, _ in seg if "mpcx_ipm_solve" in n]
            span = t1 - t0
            tot["span"] += span; tot["busy"] += busy; tot["solve"] += max(solves or [0]); tot["n"] += len(seg)
            print(f"  span {span / 1e3:7.1f} us  busy {busy / 1e3:7.1f} us  kernels {len(seg):3d}  solves "
                  + " ".join(f"{x:6.1f}" for x in solves))
        k = max(len(rs) - 1, 1)
        print(f"  mean: span {tot['span'] / k / 1e3:.1f} us, busy {tot['busy'] / k / 1e3:.1f} us, longest solve "
              f"{tot['solve'] / k:.1f} us, kernels {tot['n'] / k:.1f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1)
