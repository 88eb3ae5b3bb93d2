#!/usr/bin/env bash
# Per-rank rocprofv3 kernel traces of a multi-rank bench rehearsal on ONE GPU (ranks share cuda:0 over
# a gloo control plane).  This shell is the launcher: it never touches the GPU, and each rank process
# is rocprofv3's own child program (no exec hop behind the profiler).
#   scripts/prof_ranks.sh N [bench args...]   -> gpurun_out/prof_ranks/r<k>/..., step breakdown per rank
set -u
N=$1; shift
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_ranks
rm -rf "$OUT"; mkdir -p "$OUT"
PORT=$((20000 + RANDOM % 20000))
pids=()
for ((r = 0; r < N; r++)); do
  MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT WORLD_SIZE=$N LOCAL_WORLD_SIZE=$N RANK=$r LOCAL_RANK=$r \
  DISTRIFLOW_BACKEND=gloo HSA_ENABLE_IPC_MODE_LEGACY=0 \
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/r$r" -o k --output-format csv -- \
    python3 "$R/bench.py" --gpus "$N" "$@" > "$OUT/r$r.log" 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
for ((r = 0; r < N; r++)); do
  f=$(find "$OUT/r$r" -name '*kernel_trace.csv' | head -n 1)
  echo "== rank $r: $f"
  tail -n 2 "$OUT/r$r.log"
  [ -n "$f" ] && python3 "$R/scripts/step_breakdown.py" "$f" "${ANCHOR:-lenet_reduce}"
done
exit $rc
