#!/bin/bash
# Run a command with a heartbeat line appended to gpurun_out/heartbeat.log every 60 s, so that a long
# GPU step whose own output is sparse (first import of torch on a fresh box, long silent phases) is
# not taken for a hung one.  Exit status is the command's.
mkdir -p gpurun_out
( while sleep 60; do date +%T >> gpurun_out/heartbeat.log; done ) &
hb=$!
"$@"
rc=$?
kill $hb 2>/dev/null
exit $rc
