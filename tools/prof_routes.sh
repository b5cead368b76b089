#!/bin/bash
# rocprofv3 kernel traces and PMC passes (one counter group per run, each with
# --kernel-trace --stats only; MI355X_MICROARCH.md HBM/rocprofv3 section) of
# the three C2 routes (tools/route_probe.py: grouped / item / keyed), each run
# with its own time limit, the chain stopping at the first failure.
# usage: tools/prof_routes.sh OUT_DIR [modes]
set -o pipefail
OUT=${1:-gpurun_out/prof_routes}
MODES=${2:-"grouped item keyed"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
for m in $MODES; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/$m/trace" -o run --output-format csv \
    -- python3 "$ROOT/tools/route_probe.py" "$m" > "$ROOT/$OUT/$m.trace.log" 2>&1 || { echo "trace $m failed"; exit 1; }
  for pass in "fetch FETCH_SIZE" "write WRITE_SIZE" \
              "sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
              "sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
    set -- $pass
    name=$1; shift
    timeout -k 10 240 rocprofv3 --pmc "$@" --kernel-trace --stats -d "$ROOT/$OUT/$m/pmc/$name" -o run --output-format csv \
      -- python3 "$ROOT/tools/route_probe.py" "$m" 1000000 3 > "$ROOT/$OUT/$m.$name.log" 2>&1 || { echo "pmc $m $name failed"; exit 1; }
  done
  echo "route $m done"
done
