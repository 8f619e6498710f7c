mkdir -p gpurun_out
BEAST_LIB=tools/lib_dstep.so timeout -k 10 400 python -u -m pytest tests/test_gpu_bpe_codec.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/t_codec_dstep.log 2>&1; rc=$?; tail -2 gpurun_out/t_codec_dstep.log; [ $rc -eq 0 ] || exit $rc
BEAST_LIB=tools/lib_dstep.so timeout -k 10 300 python tools/codec/bpe_encode_run.py time > gpurun_out/enc_time_dstep.log 2>&1 || exit 3
timeout -k 10 300 python tools/codec/bpe_encode_run.py time > gpurun_out/enc_time_head.log 2>&1 || exit 4
tail -n1 gpurun_out/enc_time_dstep.log | cut -c1-100; tail -n1 gpurun_out/enc_time_head.log | cut -c1-100
