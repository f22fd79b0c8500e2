#!/bin/bash
# Local helper (this container, not the GPU box): run one gpurun call, and call it again only
# when gpurun reports that no box / slot was available or the box failed before the command
# started (status=transient: nothing ran, nothing charged).   tools/gpurun_retry.sh LOG TIMEOUT CMD
LOG=$1; T=$2; CMD=$3
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
  if grep -q "status=transient" "$LOG"; then echo "attempt $i transient" >> "$LOG.attempts"; sleep 90; continue; fi
  break
done
tail -30 "$LOG"
