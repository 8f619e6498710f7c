set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bpe_codec.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/it9_codec_tests.log 2>&1
rc=$?; echo "codec tests rc=$rc"; tail -n 30 gpurun_out/it9_codec_tests.log | grep -v "^\.\.\.\." ; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/codec/words_ab.py > gpurun_out/words_ab9.json 2> gpurun_out/words_ab9.err
rc=$?; echo "words_ab rc=$rc"; cat gpurun_out/words_ab9.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/words_ab9.err; exit $rc; }
timeout -k 10 300 python tools/codec/dw_phases.py > gpurun_out/words_phases9.json 2> gpurun_out/words_phases9.err
rc=$?; echo "phases rc=$rc"; python -c "import json; d=json.load(open('gpurun_out/words_phases9.json')); print(d['phase_us_p50_p90_p99_max']['merges'], d['row_end_us_p50_max'], d['merge_rounds_per_wave_p50_max'])"; [ $rc -eq 0 ] || exit $rc
bash tools/codec/bpe_encode_pmc.sh; rc=$?; echo "pmc rc=$rc"; cat gpurun_out/bpe_pmc/summary.json; exit $rc
