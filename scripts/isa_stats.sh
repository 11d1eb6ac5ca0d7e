# Diagnostic (CPU): compile one benchmark structure's kernel to gfx950 assembly and
# print per-function instruction / scratch / global-memory counts.
# usage: bash scripts/isa_stats.sh [model=one_room]
set -e
M=${1:-one_room}
python - "$M" <<'PY'
import sys; sys.path[:0] = ['.', 'agentlib-mpc_amd']
from agentlib_mpc_amd import benchmarks as bm
be, _ = getattr(bm, sys.argv[1])(solver_options=bm.REFERENCE)
open('/tmp/isa_model.hip', 'w').write(be.problem.gen.source)
PY
/opt/rocm/bin/hipcc --cuda-device-only -S --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Iagentlib-mpc_amd/csrc \
  /tmp/isa_model.hip -o /tmp/isa_model.s 2>&1 | grep -v hip-link || true
grep -E "^\s+\.(private_segment_fixed_size|vgpr_count|group_segment_fixed_size)" /tmp/isa_model.s | head -3
awk '/^_ZN[^ ]*: |^mpcx_ipm_solve:/{fn=$1} /scratch_store/{ss[fn]++} /scratch_load/{sl[fn]++} /global_load/{gl[fn]++} /global_store/{gs[fn]++} {n[fn]++} END{for(f in n) printf "%6d insts scr %4d/%4d glb %4d/%4d %s\n", n[f], ss[f], sl[f], gl[f], gs[f], f}' /tmp/isa_model.s | c++filt | sed 's/(.*//' | sort -k1 -n -r | head -${TOP:-14}
