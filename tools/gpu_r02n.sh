#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bpe_codec.py > gpurun_out/r02n_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/codec/bpe_encode_ab.py > gpurun_out/r02n_ab.log 2>&1
