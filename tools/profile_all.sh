#!/bin/bash
# rocprofv3 kernel trace + PMC passes for every BASELINE config's bench workload (GPU box).
# Usage: tools/profile_all.sh <tag prefix> [configs...]
set -o pipefail
P=${1:-r2}; shift || true
CFGS=${@:-c2 c3 c4 c5}
for C in $CFGS; do
  case $C in
    c2) F=65536; S=8192 ;;
    *) F=65536; S=8192 ;;
  esac
  bash tools/profile.sh ${P}_$C $C $F $S || { echo "profile $C failed"; exit 1; }
done
