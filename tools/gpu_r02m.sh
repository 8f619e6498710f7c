#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/codec/bpe_encode_phases.py run > gpurun_out/r02m_phases.json 2> gpurun_out/r02m_phases.err
