set -o pipefail
mkdir -p gpurun_out/bv
for v in _bl8 _bl16 _bl24 _bl8 _bl16 _bl24; do
  timeout -k 10 60 ./tools/beam_bench$v 64 230 500 10 > gpurun_out/bv/b$v.txt 2>&1 || exit 1
  echo "== beam_bench$v"; cat gpurun_out/bv/b$v.txt
done
