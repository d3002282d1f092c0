# bench.train_micro for the in-tree .so and every probe build tools/probes/sovar/<prefix>*.so, 2 rounds
set -o pipefail
for rep in 1 2 3; do
  for so in main tools/probes/sovar/$1*.so; do
    if [ $so = main ]; then unset APNEAUQ_SO_PATH; else export APNEAUQ_SO_PATH=$PWD/$so; fi
    echo "$rep $(basename $so .so) $(timeout -k 10 200 python -m bench.train_micro --steps 100 2>/dev/null | tail -1 | cut -c1-80)"
  done
done
