set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/it8_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -n 30 gpurun_out/it8_gpu_tests.log | grep -v "^\.\.\.\." ; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/codec/words_ab.py > gpurun_out/words_ab8.json 2> gpurun_out/words_ab8.err
rc=$?; echo "words_ab rc=$rc"; cat gpurun_out/words_ab8.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/words_ab8.err; exit $rc; }
timeout -k 10 300 python tools/codec/dw_phases.py > gpurun_out/words_phases8.json 2> gpurun_out/words_phases8.err
rc=$?; echo "phases rc=$rc"; cat gpurun_out/words_phases8.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/words_phases8.err; exit $rc; }
bash tools/ab/codec_ab.sh tools/ab/lib_ybstore.so ybstore
