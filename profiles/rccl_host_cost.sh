#!/bin/bash
# Host and GPU cost per grouped RCCL p2p exchange (profiles/calib/rccl_host_cost.cpp), one-rank communicator.
set -euo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
timeout -k 10 120 ./profiles/calib/rccl_host_cost | tee "$O/rccl_host_cost.txt"
