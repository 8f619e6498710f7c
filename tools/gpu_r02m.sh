#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bpe_codec.py tests/test_gpu_parity.py \
  -k "codec or bpe_tokenizer or api" > gpurun_out/r02m_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/codec/bpe_encode_phases.py run > gpurun_out/r02m_phases.json 2> gpurun_out/r02m_phases.err
