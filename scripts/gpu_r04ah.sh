#!/bin/bash
# round 4 (ah): the facade's per-call client lookup through a hash index
# (latency, this tree) vs the std::map alone (latency_base, the previous
# header): single-call latency at 1M clients, alternated on one box
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
for round in 1 2; do
for v in latency_base latency; do
  timeout -k 10 400 tests/cpp/$v 1048576 2000 --serve --no-oracle > gpurun_out/r04ah_$v.$round.txt 2>&1 || { tail -5 gpurun_out/r04ah_$v.$round.txt; exit 1; }
  echo "== $v $round"; tail -1 gpurun_out/r04ah_$v.$round.txt | cut -c1-300
done
done
