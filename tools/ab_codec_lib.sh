#!/bin/bash
# k_bpe_encode A/B on the GPU box: the codec GPU tests on another build of the library (BEAST_LIB),
# then the encode timing of that build and of the product.   bash tools/ab_codec_lib.sh tools/lib_x.so
LIB="$1"
mkdir -p gpurun_out
BEAST_LIB=$LIB timeout -k 10 400 python -u -m pytest tests/test_gpu_bpe_codec.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/t_codec_ab.log 2>&1; rc=$?; tail -2 gpurun_out/t_codec_ab.log; [ $rc -eq 0 ] || exit $rc
BEAST_LIB=$LIB timeout -k 10 300 python tools/codec/bpe_encode_run.py time > gpurun_out/enc_time_ab.log 2>&1 || exit 3
timeout -k 10 300 python tools/codec/bpe_encode_run.py time > gpurun_out/enc_time_product.log 2>&1 || exit 4
tail -n1 gpurun_out/enc_time_ab.log | cut -c1-100; tail -n1 gpurun_out/enc_time_product.log | cut -c1-100
