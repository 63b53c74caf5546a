#!/bin/bash
# round-5 SQ counters of the face-conv kernels (face_groups=1 so each launch is one layer over the batch)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
SQ_TAG=r7p BARGS="--steps 2 --warmup 1 --no-cpu-baseline --compare '' --host-pipeline 0 --no-timing --plates 0 --option face_groups=1" SQ_FILTER="conv|bottleneck|stem|chain" timeout -k 10 500 bash tools/runs/sq.sh
