#!/bin/bash
# interleaved A/B of two ffn2 bench binaries on one box: $1 $2 (FFN2_ANAT=2 mode, sustained)
set -o pipefail
for r in 1 2; do
  for b in "$1" "$2"; do
    echo "== $b" ; timeout -k 10 200 env FFN2_ANAT=2 ./tools/$b 32000 || exit 1
  done
done
