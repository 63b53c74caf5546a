#!/bin/bash
# PMC traffic per face-conv launch over the full batch (face_groups=1: one launch per layer, as
# the roofline's per-launch figures), fp32 headline command
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
PMC_TAG=r6pmc BARGS="--steps 2 --warmup 1 --no-cpu-baseline --compare '' --host-pipeline 0 --no-timing --option face_groups=1" timeout -k 10 700 tools/runs/pmc.sh
