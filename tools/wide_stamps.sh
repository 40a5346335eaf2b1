#!/bin/bash
# Build the WIDE_STAMPS diagnostic variant of the latency kernel (build_variants/wide_stamps) on the
# CPU; run tools/wide_stamps.py on the GPU box.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
EXTRA_FLAGS="-DWIDE_STAMPS ${EXTRA_FLAGS:-}" $ROOT/tools/build_variant.sh ${1:-wide_stamps} ${2:-$ROOT/tools/retired/br_wide_variants_r5.hip} "" br_wide
