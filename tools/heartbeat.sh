#!/bin/bash
# Prints a line every 30 s while the given command runs (long, quiet profiler passes), and returns
# the command's exit status.  usage: tools/heartbeat.sh <cmd...>
"$@" &
pid=$!
while kill -0 "$pid" 2>/dev/null; do sleep 30; kill -0 "$pid" 2>/dev/null && echo "[heartbeat] $(date +%T) $*"; done
wait "$pid"
