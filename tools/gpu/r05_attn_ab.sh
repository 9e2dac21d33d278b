#!/bin/bash
# interleaved A/B of two attention bench binaries on one box: $1 $2
set -o pipefail
for r in 1 2; do
  for b in "$1" "$2"; do
    echo "== $b" ; timeout -k 10 200 ./tools/$b 50 || exit 1
  done
done
