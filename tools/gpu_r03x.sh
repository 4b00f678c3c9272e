#!/bin/bash
# key-triple pieces at 9000 B: round size (W 12 / 8) x flush unit (48 / 24 keys)
set -e
bash tools/ab_run.sh r03x "--frame-len 9000" tri tri60 triu24 triu24w8
