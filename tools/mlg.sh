set -o pipefail
for g in 1 2 4; do
  BLS_ML_G=$g timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/mlg_$g.json 2>gpurun_out/mlg_$g.err || { tail -5 gpurun_out/mlg_$g.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/mlg_$g.json'));print($g, d['value'], d['kernels_avg_ms'])"
done
