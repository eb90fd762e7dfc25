#!/bin/bash
# Round 4 call 40: config-5 kernel trace on the final tree (8 frames) for the prefill / codec kernel split.
set -o pipefail
bash tools/prof.sh r4e_c5 --config 5 --steps 1 --warmup 0 --frames 8 > /dev/null || exit 1
echo RC=0
