set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/b1c_$i.json 2> gpurun_out/b1c_$i.err || { tail -5 gpurun_out/b1c_$i.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b1c_$i.json'));e=d['extra'];print(d['value'],e['mcd_phase_ms'],e['de_phase_ms'],e['running_bn']['value'])"
done
