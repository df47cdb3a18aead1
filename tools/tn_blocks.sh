#!/bin/bash
# TN split-K block target sweep (LLP_TN_BLOCKS) on the step's wgrad shapes.
set -e
for b in 256 512 768; do
  echo "LLP_TN_BLOCKS=$b"
  LLP_TN_BLOCKS=$b timeout -k 10 240 python tools/gemm_vs_blaslt.py
done
