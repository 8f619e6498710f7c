#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/ab/bpe_stamps.py run batch > gpurun_out/r02r_stamps0.json 2> gpurun_out/r02r_stamps.err
