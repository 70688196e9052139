#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/roles.py ${1:-32} > gpurun_out/roles${1:-32}.txt 2>&1
