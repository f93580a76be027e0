#!/bin/bash
# Optional: place the four MNIST IDX files in data/ for `--data mnist` (fpcode/init.sh downloaded them).
# This environment has no network; copy the files in by hand if you have them:
#   data/train-images-idx3-ubyte  data/train-labels-idx1-ubyte
#   data/t10k-images-idx3-ubyte   data/t10k-labels-idx1-ubyte
# Synthetic MNIST-shaped data (the default, `--data synthetic`) needs nothing.
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p data
for f in train-images-idx3-ubyte train-labels-idx1-ubyte t10k-images-idx3-ubyte t10k-labels-idx1-ubyte; do
  if [ -f "data/$f" ]; then echo "ok      data/$f"; else echo "missing data/$f"; fi
done
