set -o pipefail
mkdir -p gpurun_out/opi
for r in 1 2; do for v in "" _opi2 _opi8; do
  echo "== ffn2_bench$v" >> gpurun_out/opi/opi.txt
  timeout -k 10 120 ./tools/ffn2_bench$v 32000 >> gpurun_out/opi/opi.txt 2>&1 || exit 1
done; done
