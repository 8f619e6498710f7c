#!/bin/bash
# the whole GPU suite, one process, per-test timeout
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/suite.log 2>&1
