set -o pipefail
OUT=gpurun_out/interf; mkdir -p $OUT
for p in none hostpath keycache unique c3 msg; do
  timeout -k 10 240 python -u tools/interference_probe.py $p >> $OUT/res.jsonl 2>> $OUT/err.txt || { tail -20 $OUT/err.txt; exit 1; }
done
cat $OUT/res.jsonl
