#!/bin/bash
# round 3: measurement sets (tools/collect_r03.sh) for the given workloads, then a summary
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for WL in "$@"; do
  timeout -k 10 1000 bash tools/collect_r03.sh $WL || { echo "collect $WL failed"; exit 1; }
done
