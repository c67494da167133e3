#!/bin/bash
# Run a command with a heartbeat line appended to gpurun_out/heartbeat.log every 60 s (gpurun
# kills a command that writes nothing for 180 s; long CPU-oracle parity tests print only at
# their end).  The heartbeat stops with the command; the command's exit status is returned.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
( while sleep 60; do echo "hb $(date +%T)" >> gpurun_out/heartbeat.log; done ) &
HB=$!
"$@"
rc=$?
kill $HB 2>/dev/null
exit $rc
