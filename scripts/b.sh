#!/bin/bash
# build libfceyolo.so; on failure print the compiler output and fail
cd "$(dirname "$0")/.."
python fce-yolo_amd/build.py "$@" > /tmp/fce_build.log 2>&1 || { grep -E "error|Error" -A3 /tmp/fce_build.log | head -40; exit 1; }
tail -1 /tmp/fce_build.log
