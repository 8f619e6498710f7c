#!/bin/bash
# BPE codec on the GPU box: codec parity tests, k_bpe_encode timing per merge mode, per-row phase stamps
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_bpe_codec.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/t_codec.log 2>&1; rc=$?; tail -3 gpurun_out/t_codec.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/codec/bpe_encode_run.py time > gpurun_out/enc_time.log 2>&1 || exit 3
tail -n2 gpurun_out/enc_time.log
timeout -k 10 300 python tools/codec/bpe_encode_phases.py run gpurun_out/enc_phases.json > gpurun_out/enc_phases.log 2>&1 || exit 4
