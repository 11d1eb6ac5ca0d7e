"""LDS share, agents per CU and register budget of every structure's code objects (CPU: compile
only).  A kernel change that grows the per-agent LDS state can silently lower a structure's
agents per CU (APC is derived from the struct sizes, mpcx_ipm.hip apc_for); this lists, for the
main build of each generated source in the kernel cache, mpcx_ipm_solve's LDS bytes per
workgroup, occupancy (waves per SIMD) and scratch, so two kernel revisions can be compared.
usage: python scripts/lds_report.py [include_dir_with_mpcx_ipm.hip]  (default: the working tree)"""
import concurrent.futures as cf
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "agentlib-mpc_amd")]

from agentlib_mpc_amd.runtime import native  # noqa: E402


def one(src, inc):
    cmd = [native._hipcc(), "--cuda-device-only", "-c", "--offload-arch=gfx950", "-O3", "-std=c++17",
           f"-I{inc}", f"-I{native.INCLUDE}", f"-I{native.CSRC}", str(src), "-o", os.devnull,
           "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    m = re.search(r"Function Name: mpcx_ipm_solve(.*?)(?:Function Name|\Z)", r.stderr, re.S)
    if r.returncode != 0 or m is None:
        return src.name, "failed: " + r.stderr[-300:].replace("\n", " ")
    blk = m.group(1)
    get = lambda k: (re.search(k + r"[^:]*: (\d+)", blk) or [None, "?"])[1]  # noqa: E731
    return src.name, f"LDS {get('LDS Size')} B, occupancy {get('Occupancy')} waves/SIMD, VGPRs {get('VGPRs')}, scratch {get('ScratchSize')}"


def main():
    inc = sys.argv[1] if len(sys.argv) > 1 else str(native.CSRC)
    # the main builds' generated sources (variants differ by -D flags only); any kernel hash: the
    # generated part does not depend on it, the kernel source comes from `inc`
    seen, srcs = set(), []
    for p in sorted(native.KERNEL_DIR.glob("mpcx_*_gfx950.hip")):
        parts = p.name.split("_")
        if len(parts) == 4 and parts[1] not in seen:  # mpcx_<key>_<hash>_gfx950.hip
            seen.add(parts[1])
            srcs.append(p)
    with cf.ThreadPoolExecutor(6) as ex:
        for name, info in ex.map(lambda s: one(s, inc), srcs):
            print(f"{name:60s} {info}", flush=True)


if __name__ == "__main__":
    main()
