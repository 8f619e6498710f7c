#!/bin/bash
# GPU suite, then the host-overhead split of the B=4096 step (tools/host_overhead.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/suite.log 2>&1 &&
timeout -k 10 120 python -u tools/host_overhead.py > gpurun_out/host_overhead.log 2>&1
