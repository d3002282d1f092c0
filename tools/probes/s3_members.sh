set -o pipefail
mkdir -p gpurun_out
for st in 1 2 3 4; do
  timeout -k 10 200 python bench/train_bench.py --members 8 --streams $st --steps 20 > gpurun_out/tb_s$st.json 2> gpurun_out/tb_s$st.err || { tail -5 gpurun_out/tb_s$st.err; exit 1; }
  echo "streams $st: $(tail -1 gpurun_out/tb_s$st.json | cut -c1-300)"
done
