set -o pipefail
mkdir -p gpurun_out/pd
for r in 1 2; do for v in "" _pd5 _pd7; do
  echo "== ffn2_bench$v" >> gpurun_out/pd/pd.txt
  timeout -k 10 120 ./tools/ffn2_bench$v 32000 >> gpurun_out/pd/pd.txt 2>&1 || exit 1
done; done
