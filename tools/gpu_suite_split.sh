#!/bin/bash
# GPU suite, then the host-cost split of the B=4096 calls (tools/host_split.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/suite.log 2>&1 &&
timeout -k 10 120 python -u tools/host_split.py > gpurun_out/host_split.log 2>&1
