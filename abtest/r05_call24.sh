#!/usr/bin/env bash
# Config 5: record groups of 4 (shipped) vs 8 sparse tiles on the current kernels, alternated.
set -uo pipefail
STEPS=3 VARIANTS="rg4 rg8 rg4 rg8" bash abtest/ab_c5.sh
