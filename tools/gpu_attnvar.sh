set -o pipefail
mkdir -p gpurun_out/av
for r in 1 2; do for v in p0l0 p1l0 p0l1 p1l1; do
  echo "== $v" >> gpurun_out/av/av.txt
  timeout -k 10 120 ./tools/attn_bench_$v 20 skipx6 >> gpurun_out/av/av.txt 2>&1 || exit 1
done; done
