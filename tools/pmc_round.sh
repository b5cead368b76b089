#!/bin/bash
# PMC passes over the bench command (one counter group per rocprofv3 run, each
# with --kernel-trace --stats only, as MI355X_MICROARCH.md prescribes: FETCH_SIZE
# and WRITE_SIZE cannot share a pass).  Each pass has its own time limit and the
# chain stops at the first failure.  Summaries: tools/pmc_summary.py.
set -o pipefail
OUT=${1:-gpurun_out/pmc}
N=${2:-1000000}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > "$ROOT/$OUT/counters_list.txt" 2>&1 || true
BENCH=("$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-latency --no-extras --items "$N")
if [ "${MODE:-secp}" = ed ]; then BENCH=("$ROOT/tools/ed_probe.py" "$N" 16); fi   # ed25519 kernels
if [ "${MODE:-secp}" = item ]; then BENCH+=(--keys "$N"); fi                           # per-item route: every key distinct
if [ "${MODE:-secp}" = kw ]; then BENCH=("$ROOT/tools/kw_pmc_probe.py"); fi          # the resident arena's wide-window ladder
if [ "${MODE:-secp}" = lat ]; then BENCH=("$ROOT/tools/lat_pmc_probe.py"); fi        # sliced small-batch kernels
pass() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --stats -d "$ROOT/$OUT/$name" -o run --output-format csv \
    -- python3 "${BENCH[@]}" > "$ROOT/$OUT/$name.json" 2> "$ROOT/$OUT/$name.err" \
    || { echo "pass $name failed"; tail -20 "$ROOT/$OUT/$name.err"; return 1; }
  echo "pass $name ok"
}
pass fetch FETCH_SIZE &&
pass write WRITE_SIZE &&
pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE &&
pass sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
