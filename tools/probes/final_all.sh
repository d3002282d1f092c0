set -o pipefail
bash tools/probes/final_check.sh || exit 1
timeout -k 10 200 python -m bench.train_micro --steps 100 2>/dev/null | tail -1
timeout -k 10 200 python bench/train_bench.py --members 8 --streams 3 --steps 20 2>/dev/null | tail -1 | cut -c1-200
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { tail -5 gpurun_out/final_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/final_bench.json'));e=d['extra'];print(d['value'],e['mcd_phase_ms'],e['de_phase_ms'],e['running_bn']['value'])"
