set -o pipefail
cd "$GRAFT_REPO_ROOT"
for pk in 0 1024; do
  if [ $pk = 0 ]; then unset SH_PART_KEYS; else export SH_PART_KEYS=$pk; fi
  timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 3 > gpurun_out/c4pk_$pk.json 2>/dev/null || { echo "c4 $pk failed"; exit 1; }
  echo "pk=$pk $(python3 -c "import json;d=json.load(open('gpurun_out/c4pk_$pk.json'));print(d['value'], d['ms_per_step'])")"
done
