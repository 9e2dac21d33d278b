set -o pipefail
mkdir -p gpurun_out/nbt
for r in 1 2; do for v in "" _nbt2; do
  echo "== ffn2_bench$v" >> gpurun_out/nbt/nbt.txt
  timeout -k 10 120 ./tools/ffn2_bench$v 32000 >> gpurun_out/nbt/nbt.txt 2>&1 || exit 1
done; done
