set -o pipefail
mkdir -p gpurun_out/bv
for v in "" _v4 "" _v4; do
  timeout -k 10 60 ./tools/beam_bench$v 64 230 500 10 > gpurun_out/bv/b$v.txt 2>&1 || exit 1
  echo "== beam_bench$v"; head -3 gpurun_out/bv/b$v.txt; grep "scores sum" gpurun_out/bv/b$v.txt
done
