set -o pipefail
mkdir -p gpurun_out
for ms in 262144 524288 1048576 262144; do
  APNEAUQ_MCD_MAX_SAMPLES=$ms timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-secondary --no-deviation > gpurun_out/chunk_$ms.json 2>gpurun_out/chunk_$ms.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/chunk_$ms.json'));print($ms, d['value'], d['extra']['mcd_phase_ms'], d['extra']['de_phase_ms'])"
done
