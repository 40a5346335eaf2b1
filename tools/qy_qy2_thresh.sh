#!/bin/bash
# qy (kind 4) against qy2 (kind 5) of the product build at the sizes around the engine's switch
# (Context::kQy2Min), fresh process per run (tools/qy2_probe.py).
set -u
for r in 1 2; do
  for B in 1024 2048 2560 3072; do
    for K in 4 5; do timeout -k 10 120 python -u tools/qy2_probe.py fhe-sign_amd $K $B 3 || exit $?; done
  done
done
