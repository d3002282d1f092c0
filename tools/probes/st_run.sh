export PYTHONPATH=$PWD
for v in 0 4 16 20; do APNEAUQ_SO_PATH=$PWD/tools/probes/sovar/st4_$v.so timeout -k 10 120 python3 tools/probes/fwd_stamps.py > gpurun_out/st4_$v.json 2> gpurun_out/st4_$v.err || exit 1; echo "== $v"; python3 -c "import json;d=json.load(open('gpurun_out/st4_$v.json'));print(d['median_cycles'],d['median_tile'],round(d['frac_of_conv_overlapping_partner_conv'],2))"; done
bash tools/gpu_iter.sh r2b tests/test_prep_gpu.py tests/test_train_gpu.py tests/test_deterministic_gpu.py tests/test_generic_train_gpu.py tests/test_fused_gpu.py
