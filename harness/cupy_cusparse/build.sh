#!/usr/bin/env bash
# Port of cupy_cusparse/build.sh: builds the three native drivers against libmi355_spgemm.so
set -e
make -C "$(cd "$(dirname "${BASH_SOURCE[0]}")/../.." && pwd)" lib drivers
echo "Compile Finish"
