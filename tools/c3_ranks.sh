#!/bin/bash
# All of C3 on one GPU, one rank at a time: rank r of 8 scans its 128 GiB of
# the 1 TiB seed-3 volume, cuts from its true entry (the golden exit of rank
# r-1) and hashes; each line's exact.golden_match checks the rank's chunk list
# against tests/golden/full_configs.json.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
for r in 0 1 2 3 4 5 6 7; do
  bash tools/gpu.sh bench "c3r$r" --share "$r/8" --steps 2 --warmup 1 || exit $?
done
