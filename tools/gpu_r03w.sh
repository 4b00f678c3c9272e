#!/bin/bash
# key-triple pieces: round fill at 9000 B (lines policy carries up to 47 keys per bucket)
set -e
bash tools/ab_run.sh r03w "--frame-len 9000" tri tri85 tri80 tri72
