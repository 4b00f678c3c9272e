#!/bin/bash
set -e
mkdir -p gpurun_out
bash tools/bimodal.sh r03e 4 > gpurun_out/bimodal_r03e.txt 2>&1
