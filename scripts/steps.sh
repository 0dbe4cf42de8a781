#!/bin/bash
# One gpurun call made of named GPU steps, each under its own time limit; the first failure ends
# the call (a timeout, signal or crash must not be followed by more GPU work).
#   bash scripts/steps.sh TAG "name|seconds|command" ["name|seconds|command" ...]
# Each step's stdout+stderr goes to gpurun_out/TAG_name.log; its last lines are echoed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
for S in "$@"; do
  NAME=${S%%|*}; REST=${S#*|}; SECS=${REST%%|*}; CMD=${REST#*|}
  LOG=gpurun_out/${TAG}_${NAME}.log
  echo "== $NAME ($SECS s): $CMD"
  timeout -k 10 "$SECS" bash -c "$CMD" > "$LOG" 2>&1
  rc=$?
  tail -${TAIL:-6} "$LOG"
  [ $rc -ne 0 ] && { echo "step $NAME failed rc=$rc"; exit $rc; }
done
exit 0
