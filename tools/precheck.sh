#!/bin/bash
# Build everything and run the CPU suite; a GPU call should only follow a clean precheck.
set -e
cd "$(dirname "$0")/.."
make -s -j8 -C storage-engines_amd/csrc
make -s -C storage-engines_amd/harness
make -s -C oracle
python -m pytest tests -q -m "not gpu" -x 2>&1 | tail -1
